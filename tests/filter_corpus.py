"""Partition-pruning corpora for the K5 tests: a table whose partition values exercise Spark's
non-ANSI Cast(string AS type) edge cases (whitespace, signs, leading zeros, overflow, bad dates,
boolean spellings, nulls, JSON escapes, non-ASCII), written as JSON commits and, optionally, as a
checkpoint of the same state followed by more commits."""
import json
import os

from delta_amd.testing import synth as S

SCHEMA = {"type": "struct", "fields": [
    {"name": "id", "type": "long", "nullable": True, "metadata": {}},
    {"name": "part", "type": "integer", "nullable": True, "metadata": {}},
    {"name": "d", "type": "date", "nullable": True, "metadata": {}},
    {"name": "b", "type": "boolean", "nullable": True, "metadata": {}},
    {"name": "s", "type": "string", "nullable": True, "metadata": {}},
    {"name": "big", "type": "long", "nullable": True, "metadata": {}},
]}
PCOLS = ["part", "d", "b", "s", "big"]
METADATA = {"id": "filter-corpus", "format": {"provider": "parquet", "options": {}},
            "schemaString": json.dumps(SCHEMA, separators=(",", ":")), "partitionColumns": PCOLS,
            "configuration": {}, "createdTime": 1600000000000}
PROTOCOL = {"minReaderVersion": 1, "minWriterVersion": 2}

PART = ["3", " 3", "+3", "03", "3.0", "", None, "abc", "2147483648", "-2147483648", "1", "2", "4", "-7", "\t5\n"]
DATE = ["2020-03-01", "2020-3-1", "2020-03-01 12:00:00", "2020", "2020-02-30", "20200301", None, "2020-05-31",
        "2020-06-01", "2019-12-31T23:59", " 2020-04-15 ", "2020-13-01", "2020-02-29", "2021-02-29"]
BOOL = ["true", "TRUE", "yes", "0", "maybe", None, "f", "N", " t "]
STR = ["w17", "w1", "", None, 'a"b', "été", "w\\1", "w17 ", "W17", "a/b"]
BIG = ["9223372036854775807", "9223372036854775808", "-9223372036854775808", "12", None, "1e3"]


def _pv(i):
    # strides coprime with the list lengths: every value of every column occurs
    return {"part": PART[i % len(PART)], "d": DATE[(i * 3 + 1) % len(DATE)], "b": BOOL[(i * 2 + 1) % len(BOOL)],
            "s": STR[(i * 7) % len(STR)], "big": BIG[(i * 5) % len(BIG)]}


def _add(i, pv=None):
    return {"path": "f-%05d.parquet" % i, "partitionValues": pv if pv is not None else _pv(i), "size": 100 + i,
            "modificationTime": 1600000000000 + i, "dataChange": True, "stats": None}


def _line(a):
    return json.dumps(a, separators=(",", ":"), ensure_ascii=bool(len(str(a)) % 2))  # mix raw / \\u escapes


def build(table_dir, n=600, checkpoint=False, escaped_keys=False):
    """Returns the _delta_log path. Commits: v0 protocol+metadata+adds[0:n/2], v1 removes some and
    adds [n/2:n]; with `checkpoint`, a checkpoint of the v1 state and v2 adding a few more."""
    log = os.path.join(table_dir, "_delta_log")
    os.makedirs(log, exist_ok=True)
    h = n // 2
    v0 = [{"protocol": PROTOCOL}, {"metaData": METADATA}] + [{"add": _add(i)} for i in range(h)]
    if escaped_keys:  # a map key written with a JSON escape still names the column
        v0.append({"add": _add(n + 1, {"p\\u0061rt": "3"})})
    with open(os.path.join(log, "%020d.json" % 0), "w") as f:
        for a in v0:
            f.write(_line(a).replace("p\\\\u0061rt", "p\\u0061rt") + "\n")
    removed = list(range(0, h, 9))
    v1 = [{"remove": {"path": "f-%05d.parquet" % i, "deletionTimestamp": 1600000001000, "dataChange": True}}
          for i in removed] + [{"add": _add(i)} for i in range(h, n)]
    with open(os.path.join(log, "%020d.json" % 1), "w") as f:
        for a in v1:
            f.write(_line(a) + "\n")
    if checkpoint:
        live = [_add(i) for i in range(n) if i not in set(removed)]
        if escaped_keys:
            live.append(_add(n + 1, {"part": "3"}))
        S.write_checkpoint_records(os.path.join(log, "%020d.checkpoint.parquet" % 1), PROTOCOL, METADATA, live,
                                   row_group_size=200, use_dictionary=True)
        with open(os.path.join(log, "_last_checkpoint"), "w") as f:
            f.write('{"version":1,"size":%d}\n' % (len(live) + 2))
        with open(os.path.join(log, "%020d.json" % 2), "w") as f:
            for i in range(n + 10, n + 40):
                f.write(_line({"add": _add(i)}) + "\n")
    return log


C = lambda n: ("col", n)  # noqa: E731
L = lambda t, v: ("lit", t, v)  # noqa: E731

PREDICATES = [
    [("=", C("part"), L("integer", 3))],
    [("in", C("part"), [L("integer", 1), L("integer", 3)])],
    [("in", C("part"), [L("integer", 1), L("integer", None)])],
    [("not", ("in", C("part"), [L("integer", 1), L("integer", 3)]))],
    [(">=", C("part"), L("integer", 2))],
    [(">", C("part"), L("integer", 1)), ("<=", C("part"), L("integer", 3))],
    [("or", (">=", C("part"), L("integer", 3)), ("<", C("part"), L("integer", 0)))],
    [("isnull", C("part"))],
    [("isnotnull", C("PART"))],
    [(">=", C("d"), L("date", "2020-03-01")), ("<", C("d"), L("date", "2020-06-01"))],
    [("=", C("d"), L("date", "2020-02-29"))],
    [("isnull", C("d"))],
    [("=", C("b"), L("boolean", True))],
    [("not", ("=", C("b"), L("boolean", True)))],
    [("<=>", C("b"), L("boolean", None))],
    [("=", C("s"), L("string", "w17"))],
    [("<", C("s"), L("string", "w"))],
    [("!=", C("s"), L("string", "w17"))],
    [("<=>", C("s"), L("string", None))],
    [("=", C("s"), L("string", 'a"b'))],
    [("=", C("s"), L("string", "été"))],
    [(">", C("big"), L("long", 0))],
    [("=", C("big"), L("long", -9223372036854775808))],
    [("and", ("=", C("part"), L("integer", 3)), ("=", C("b"), L("boolean", True)))],
    [("or", (">=", C("part"), L("integer", 1)), (">", C("d"), L("date", "2020-05-01")))],
    # literal first (the leaf form flips the comparison), string IN sets with a NULL, NOT IN with a
    # NULL (never true), a column-vs-column comparison (the generic interpreter in either mode)
    [("<", L("integer", 2), C("part"))],
    [(">=", L("date", "2020-04-15"), C("d"))],
    [("in", C("s"), [L("string", "w17"), L("string", "été"), L("string", None), L("string", "w1")])],
    [("not", ("in", C("part"), [L("integer", 4), L("integer", None)]))],
    [("=", C("part"), C("part"))],
    [("and", ("or", ("isnull", C("s")), ("=", C("b"), L("boolean", False))), ("not", ("<", C("big"), L("long", 1))))],
]
