"""Host-side logic of the product that needs no GPU: interval rendering for the reference's
retention-policy error text."""
from delta_amd.delta_log import calendar_interval, interval_to_string, retention_text


def test_calendar_interval_rendering():
    # CalendarInterval.toString of what DeltaConfigs.parseCalendarInterval reads from a property
    assert interval_to_string(*calendar_interval("interval 30 days")) == "30 days"
    assert interval_to_string(*calendar_interval("interval 1 week")) == "7 days"
    assert interval_to_string(*calendar_interval("interval 36 hours")) == "36 hours"
    assert interval_to_string(*calendar_interval("INTERVAL 1 day 90 minutes")) == "1 days 1 hours 30 minutes"
    assert interval_to_string(*calendar_interval("interval 2500 milliseconds")) == "2.5 seconds"
    assert interval_to_string(0, 0, 0) == "0 seconds"


def test_retention_text_defaults_and_table_values():
    assert retention_text(None) == ("(delta.logRetentionDuration=30 days) and checkpoint retention policy "
                                    "(delta.checkpointRetentionDuration=2 days)")
    md = {"configuration": {"delta.checkpointRetentionDuration": "interval 3 days"}}
    assert retention_text(md).endswith("(delta.checkpointRetentionDuration=3 days)")
