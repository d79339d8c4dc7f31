"""Action.fromJson and DeltaLog.getChanges, host side.

Expected values restate the reference's serializer tests (T/ActionSerializerSuite.scala:94-124)
and getChanges' contract (D/DeltaLog.scala:222-238) over the reference's golden logs.
"""
import os
import shutil

import pytest

from delta_amd.actions import DataLossError, data_loss_message, from_json, get_changes
from tests.conftest import GOLDEN

LOG020 = os.path.join(GOLDEN, "ref", "delta-0.2.0", "_delta_log")


def test_remove_file_defaults():
    # T/ActionSerializerSuite.scala:94-104: Jackson ignores Scala defaults (dataChange -> false)
    base = {"path": "a", "extendedFileMetadata": False, "partitionValues": None, "size": 0, "tags": None}
    assert from_json('{"remove":{"path":"a","deletionTimestamp":2,"dataChange":true}}') == \
        {"remove": dict(base, deletionTimestamp=2, dataChange=True)}
    assert from_json('{"remove":{"path":"a","dataChange":false}}') == \
        {"remove": dict(base, deletionTimestamp=None, dataChange=False)}
    assert from_json('{"remove":{"path":"a","deletionTimestamp":5}}') == \
        {"remove": dict(base, deletionTimestamp=5, dataChange=False)}


def test_extra_fields_and_txn():
    # "extra fields" (:121-124) and the SetTransaction round trips (:106-110)
    assert from_json('{"txn": {"test": 1}}') == {"txn": {"appId": None, "version": 0, "lastUpdated": None}}
    assert from_json('{"txn":{"appId":"a","version":1,"lastUpdated":1234}}') == \
        {"txn": {"appId": "a", "version": 1, "lastUpdated": 1234}}
    assert from_json('{"txn":{"appId":"a","version":1}}') == {"txn": {"appId": "a", "version": 1, "lastUpdated": None}}


def test_unwrap_priority_and_nulls():
    assert from_json('{"commitInfo":{"x":1},"add":{"path":"p","size":3}}')["add"]["size"] == 3
    assert list(from_json('{"protocol":{"minReaderVersion":1},"txn":{"appId":"t"}}')) == ["txn"]
    assert from_json('{"add":null,"remove":null}') is None
    assert from_json('{}') is None
    assert from_json('{"protocol":{}}') == {"protocol": {"minReaderVersion": 0, "minWriterVersion": 0}}
    assert from_json('{"add":{"path":"p","size":"12","modificationTime":1.9,"dataChange":1}}')["add"] == {
        "path": "p", "partitionValues": None, "size": 12, "modificationTime": 1, "dataChange": True,
        "stats": None, "tags": None}
    for bad in ('{"add":{"size":"x"}}', '{"add":[]}', "[1]", "{", '{"add":{"size":NaN}}'):
        with pytest.raises(ValueError):
            from_json(bad)


def test_get_changes_golden():
    kinds = [(v, [next(iter(a)) for a in acts]) for v, acts in get_changes(LOG020, 0)]
    assert [v for v, _ in kinds] == [0, 1, 2, 3]
    assert kinds[3][1] == ["commitInfo", "txn", "add"]
    assert sum(k == "remove" for _, ks in kinds for k in ks) == 4
    assert [v for v, _ in get_changes(LOG020, 2)] == [2, 3]
    assert list(get_changes(LOG020, 10)) == []
    rm = [a["remove"] for _, acts in get_changes(LOG020, 2) for a in acts if "remove" in a]
    assert {r["deletionTimestamp"] for r in rm} == {1564524298213, 1564524298214}


def test_get_changes_fail_on_data_loss(tmp_path):
    log = tmp_path / "_delta_log"
    shutil.copytree(LOG020, log)
    os.remove(log / ("%020d.json" % 1))
    assert [v for v, _ in get_changes(str(log), 0)] == [0, 2, 3]
    with pytest.raises(DataLossError) as ei:
        list(get_changes(str(log), 0, fail_on_data_loss=True))
    assert str(ei.value) == data_loss_message(1, 2)
    assert str(ei.value).startswith("The stream from your Delta table was expecting process data from version 1,\n"
                                    "but the earliest available version in the _delta_log directory is 2.")
    assert [v for v, _ in get_changes(str(log), 2, fail_on_data_loss=True)] == [2, 3]
