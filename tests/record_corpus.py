"""A log whose survivors exercise every field of the full-record checksum (oracle.delta_oracle
.record_hash): a checkpoint (the reference's column layout, tests' pyarrow writer) with tags, null and
empty maps, escaped / non-ASCII stats and removes with and without deletionTimestamp and
extendedFileMetadata, then JSON commits with repeated members and map keys, absent primitives, JSON
nulls and escapes, removes of checkpoint paths and re-adds. Built from data only (no reference
source); the expected sums come from the Python oracle."""
import json
import os

PROTOCOL = {"minReaderVersion": 1, "minWriterVersion": 2}
METADATA = {"id": "rec-corpus", "format": {"provider": "parquet", "options": {}},
            "schemaString": json.dumps({"type": "struct", "fields": [
                {"name": "p", "type": "string", "nullable": True, "metadata": {}},
                {"name": "q", "type": "integer", "nullable": True, "metadata": {}}]}),
            "partitionColumns": ["p", "q"], "configuration": {}, "createdTime": 1}


def _ck_rows():
    adds, removes = [], []
    for i in range(40):
        adds.append({"path": "p=%d/q=%d/part-%05d.parquet" % (i % 3, i % 5, i),
                     "partitionValues": None if i % 13 == 7 else ({} if i % 11 == 5 else
                                                                  {"p": str(i % 3), "q": None if i % 4 == 0 else str(i % 5)}),
                     "size": 1000 + i * 37, "modificationTime": 1_600_000_000_000 + i,
                     "tags": None if i % 2 else {"ZCUBE": "z%d" % i, "INSERTION_TIME": str(i)},
                     "stats": None if i % 5 == 0 else '{"numRecords":%d,"minValues":{"s":"\\u00e9\\"x%d"}}' % (i, i)})
    for i in range(12):
        removes.append({"path": "gone/part-%05d.parquet" % i,
                        "deletionTimestamp": None if i % 3 == 0 else 1_600_000_100_000 + i,
                        "dataChange": True, "extendedFileMetadata": bool(i % 2),
                        "partitionValues": None if i % 4 == 0 else {"p": "r%d" % i},
                        "size": 0 if i % 5 == 0 else 50 + i, "tags": {"t": None} if i == 3 else None})
    return adds, removes


def build(table: str) -> str:
    """Writes the table; returns its _delta_log path."""
    from delta_amd.testing import synth as S
    lp = os.path.join(table, "_delta_log")
    os.makedirs(lp, exist_ok=True)
    adds, removes = _ck_rows()
    S.write_checkpoint_records(os.path.join(lp, "%020d.checkpoint.parquet" % 5), PROTOCOL, METADATA, adds, removes,
                               row_group_size=16)
    with open(os.path.join(lp, "_last_checkpoint"), "w") as f:
        f.write('{"version":5,"size":%d}\n' % (len(adds) + len(removes) + 2))
    lines6 = [
        # repeated member: the last "size" and "partitionValues" win; a repeated map key keeps its last value
        '{"add":{"path":"j/a","partitionValues":{"p":"x"},"size":1,"size":2,"modificationTime":3,'
        '"dataChange":true,"partitionValues":{"p":"y","q":"1","p":"z"},"stats":"{\\"n\\":1}"}}',
        # absent size / modificationTime read 0; JSON null stats / tags
        '{"add":{"path":"j/b","partitionValues":{"p":null},"dataChange":false,"stats":null,"tags":null}}',
        # escapes in the path, values, tags
        '{"add":{"path":"j/c%20d\\u00e9","partitionValues":{"p":"\\t\\"q\\""},"size":9,"modificationTime":-4,'
        '"dataChange":true,"tags":{"k\\u0031":"v","e":""}}}',
        # remove of checkpoint adds (one tombstone kept, one without a deletionTimestamp)
        '{"remove":{"path":"p=1/q=1/part-00001.parquet","deletionTimestamp":1600000200000,"dataChange":true,'
        '"extendedFileMetadata":true,"partitionValues":{"p":"1","q":"1"},"size":1037}}',
        '{"remove":{"path":"p=2/q=2/part-00002.parquet","dataChange":true}}',
        '{"commitInfo":{"timestamp":1}}',
    ]
    lines7 = [
        # re-add of a removed checkpoint path, with a different record
        '{"add":{"path":"p=1/q=1/part-00001.parquet","partitionValues":{"p":"1","q":"1"},"size":77,'
        '"modificationTime":8,"dataChange":false,"stats":"{}"}}',
        # remove of a JSON add with tags and an empty map
        '{"remove":{"path":"j/b","deletionTimestamp":1600000300000,"dataChange":true,"partitionValues":{},'
        '"size":3,"tags":{"a":"b"}}}',
        # a tombstone of a checkpoint remove replaced by a newer one
        '{"remove":{"path":"gone/part-00004.parquet","deletionTimestamp":1600000400000,"dataChange":false,'
        '"extendedFileMetadata":false,"size":5}}',
    ]
    for v, lines in ((6, lines6), (7, lines7)):
        with open(os.path.join(lp, "%020d.json" % v), "w") as f:
            f.write("\n".join(lines) + "\n")
    return lp


CUTOFFS = (0, 1_600_000_100_005)
