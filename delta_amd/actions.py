"""Driver-side action decoding: `Action.fromJson` and `DeltaLog.getChanges`.

`Action.fromJson` (D/actions/actions.scala:57-59) is Jackson (`JsonUtils.mapper`,
D/util/JsonUtils.scala:26-31: unknown properties ignored, DefaultScalaModule) reading a
`SingleAction` and unwrapping it with priority add > remove > metaData > txn > protocol > cdc >
commitInfo (D/actions/actions.scala:523-541). Jackson does not apply Scala default arguments:
an absent `Long`/`Int` reads 0, an absent `Boolean` false, an absent `String`/`Map` null and an
absent `Option` None — `{"remove":{"path":"a","deletionTimestamp":5}}` is a RemoveFile with
dataChange=false (T/ActionSerializerSuite.scala:94-104). Scalars are coerced the way Jackson's
defaults do (numeric strings to numbers, fractions truncated, 0/1 to booleans); a value Jackson
cannot coerce raises `ValueError`, as `readValue` throws.

The GPU replay path (K1, k_json.hip) reads the same lines for the state; this module materialises
full Action records for the streaming tail (`getChanges`), which the reference also decodes on
the driver. Parity is pinned on the file actions, txn and protocol (the reference's serializer
tests); metaData / commitInfo / cdc records are returned with their fields as written (the
absent-field defaults of those case classes are parity unpinned).
"""
import json
import os
import re
from typing import Iterator, List, Optional, Tuple

ORDER = ("add", "remove", "metaData", "txn", "protocol", "cdc", "commitInfo")

# field -> kind: "long" | "int" | "bool" | "str" | "map" | "optlong"
ADD_FIELDS = {"path": "str", "partitionValues": "map", "size": "long", "modificationTime": "long",
              "dataChange": "bool", "stats": "str", "tags": "map"}           # D/actions/actions.scala:220-230
REMOVE_FIELDS = {"path": "str", "deletionTimestamp": "optlong", "dataChange": "bool",
                 "extendedFileMetadata": "bool", "partitionValues": "map", "size": "long",
                 "tags": "map"}                                                  # :307-316
CDC_FIELDS = {"path": "str", "partitionValues": "map", "size": "long", "tags": "map"}  # :325-330
TXN_FIELDS = {"appId": "str", "version": "long", "lastUpdated": "optlong"}    # :197-203
PROTOCOL_FIELDS = {"minReaderVersion": "int", "minWriterVersion": "int"}      # :81-84
SCHEMAS = {"add": ADD_FIELDS, "remove": REMOVE_FIELDS, "cdc": CDC_FIELDS, "txn": TXN_FIELDS,
           "protocol": PROTOCOL_FIELDS}

_DELTA = re.compile(r"^(\d{20})\.json$")  # FileNames.deltaFilePattern (D/util/FileNames.scala:25)


def _integral(v, bits: int) -> int:
    if isinstance(v, bool):
        raise ValueError("boolean for a numeric field")
    if isinstance(v, str):
        try:
            v = float(v) if any(c in v for c in ".eE") else int(v)
        except ValueError:
            raise ValueError("cannot coerce %r to a number" % v)
    if isinstance(v, float):
        if v != v or abs(v) >= 2.0 ** (bits - 1):
            raise ValueError("numeric value out of range")
        v = int(v)  # ACCEPT_FLOAT_AS_INT truncates
    if not isinstance(v, int):
        raise ValueError("cannot coerce %r to a number" % (v,))
    if not -(1 << (bits - 1)) <= v < (1 << (bits - 1)):
        raise ValueError("numeric value out of range")
    return v


def _field(kind: str, v):
    if kind in ("long", "int"):
        return 0 if v is None else _integral(v, 64 if kind == "long" else 32)
    if kind == "optlong":
        return None if v is None else _integral(v, 64)
    if kind == "bool":
        if v is None:
            return False
        if isinstance(v, bool):
            return v
        if isinstance(v, int) and not isinstance(v, bool):
            return v != 0
        if isinstance(v, str) and v in ("true", "false"):
            return v == "true"
        raise ValueError("cannot coerce %r to a boolean" % (v,))
    if kind == "str":
        if v is None or isinstance(v, str):
            return v
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            return json.dumps(v)  # scalar coerced to its text
        if isinstance(v, bool):
            return "true" if v else "false"
        raise ValueError("cannot coerce %r to a string" % (v,))
    # map<string,string>
    if v is None:
        return None
    if not isinstance(v, dict):
        raise ValueError("cannot coerce %r to a map" % (v,))
    return {k: _field("str", x) for k, x in v.items()}


def from_json(line: str) -> Optional[dict]:
    """Action.fromJson: the unwrapped action as {"<kind>": {fields}}, or None when every action
    field of the SingleAction is null. Raises ValueError for input Jackson rejects."""
    try:
        obj = json.loads(line, parse_constant=lambda s: (_ for _ in ()).throw(ValueError(s)))
    except json.JSONDecodeError as e:
        raise ValueError("malformed action: %s" % e)
    if not isinstance(obj, dict):
        raise ValueError("an action must be a JSON object")
    for name in ORDER:
        v = obj.get(name)
        if v is None:
            continue
        if not isinstance(v, dict):
            raise ValueError("%s must be an object" % name)
        schema = SCHEMAS.get(name)
        if schema is None:
            return {name: v}
        return {name: {f: _field(k, v.get(f)) for f, k in schema.items()}}
    return None


class DataLossError(Exception):
    """DeltaErrors.failOnDataLossException (D/DeltaErrors.scala:221-233): IllegalStateException."""

    kind = "IllegalStateException"


def data_loss_message(expected: int, seen: int) -> str:
    return ("The stream from your Delta table was expecting process data from version %d,\n"
            "but the earliest available version in the _delta_log directory is %d. The files\n"
            "in the transaction log may have been deleted due to log cleanup. In order to avoid losing\n"
            "data, we recommend that you restart your stream with a new checkpoint location and to\n"
            "increase your delta.logRetentionDuration setting, if you have explicitly set it below 30\n"
            "days.\n"
            "If you would like to ignore the missed data and continue your stream from where it left\n"
            "off, you can set the .option(\"failOnDataLoss\", \"false\") as part\n"
            "of your readStream statement.\n       " % (expected, seen))  # the literal's last line


def get_changes(log_path: str, start_version: int, fail_on_data_loss: bool = False
                ) -> Iterator[Tuple[int, List[Optional[dict]]]]:
    """DeltaLog.getChanges (D/DeltaLog.scala:222-238): every delta file at or after
    `start_version`, in version order, as (version, [Action.fromJson(line) ...])."""
    start = "%020d.json" % start_version
    names = sorted(n for n in (os.listdir(log_path) if os.path.isdir(log_path) else []) if n >= start)
    last_seen = start_version - 1
    for n in names:
        m = _DELTA.match(n)
        if not m:
            continue
        version = int(m.group(1))
        if fail_on_data_loss and version > last_seen + 1:
            raise DataLossError(data_loss_message(last_seen + 1, version))
        last_seen = version
        with open(os.path.join(log_path, n), "r", encoding="utf-8") as f:
            lines = f.read().split("\n")
        if lines and lines[-1] == "":
            lines.pop()  # the file's final newline ends the last line
        yield version, [from_json(l) for l in lines]
