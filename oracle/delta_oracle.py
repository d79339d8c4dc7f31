"""CPU restatement of Delta Lake snapshot state reconstruction -- TEST INFRASTRUCTURE ONLY.

This module is the *oracle*: a plain-Python restatement of the reference's replay path used
by `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg as the checker.
The product (`delta_amd`, `libdeltareplay.so`) never imports it.

Parity pin: validated in `tests/test_oracle_golden.py` against the reference's own fixtures
(`tests/golden/ref`, copied data from `core/src/test/resources/delta/`): the delta-0.2.0
checkpoint is the reference's replay of its JSON v0..v3; delta-0.1.0 likewise modulo the old
writer's dataChange; the dbr_8_* `.crc` files pin the computedState aggregates.

Citations are relative to the reference checkout; `D/` = core/src/main/scala/org/apache/spark/
sql/delta/.
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

# ----------------------------------------------------------------------------------------------
# FileNames (D/util/FileNames.scala:25-107)
# ----------------------------------------------------------------------------------------------
_DELTA_RE = re.compile(r"^\d+\.json$")
_CKPT_RE = re.compile(r"^\d+\.checkpoint(\.\d+\.\d+)?\.parquet$")
_CRC_RE = re.compile(r"^\d+\.crc$")


def delta_file(version: int) -> str:  # D/util/FileNames.scala:33
    return "%020d.json" % version


def checkpoint_file_singular(version: int) -> str:  # :55
    return "%020d.checkpoint.parquet" % version


def checkpoint_file_with_parts(version: int, num_parts: int) -> List[str]:  # :70-73
    return ["%020d.checkpoint.%010d.%010d.parquet" % (version, i, num_parts)
            for i in range(1, num_parts + 1)]


def is_delta_file(name: str) -> bool:  # :83
    return bool(_DELTA_RE.match(name))


def is_checkpoint_file(name: str) -> bool:  # :81
    return bool(_CKPT_RE.match(name))


def num_checkpoint_parts(name: str) -> Optional[int]:  # :75-79
    seg = name.split(".")
    return None if len(seg) != 5 else int(seg[3])


def file_version(name: str) -> int:  # :93-107 (delta/checkpoint/crc all lead with the version)
    return int(name.split(".")[0])


# ----------------------------------------------------------------------------------------------
# CheckpointInstance / LogSegment (D/Checkpoints.scala:60-106,210-218;
# D/SnapshotManagement.scala:82-179,365-372,394-416)
# ----------------------------------------------------------------------------------------------
class DeltaError(Exception):
    """Mirrors the reference's exception classes by `kind` (D/DeltaErrors.scala)."""

    def __init__(self, kind: str, msg: str):
        super().__init__(msg)
        self.kind = kind


@dataclass(frozen=True)
class CheckpointInstance:
    version: int
    num_parts: Optional[int]

    def sort_key(self):  # compare(): version, then parts (None counts as 1)
        return (self.version, 1 if self.num_parts is None else self.num_parts)

    def files(self) -> List[str]:
        if self.num_parts is None:
            return [checkpoint_file_singular(self.version)]
        return checkpoint_file_with_parts(self.version, self.num_parts)


@dataclass
class LogSegment:
    log_path: str
    version: int
    deltas: List[str]            # file names, ascending version
    checkpoint: List[str]        # file names of the chosen checkpoint's parts
    checkpoint_version: Optional[int]


def read_last_checkpoint(log_path: str) -> Optional[dict]:
    """Checkpoints.lastCheckpoint (D/Checkpoints.scala:148-175) minus the retry sleeps: a
    corrupt file falls back to listing (findLastCompleteCheckpoint)."""
    p = os.path.join(log_path, "_last_checkpoint")
    if not os.path.exists(p):
        return None
    try:
        with open(p, "r") as f:
            line = f.readline()
        d = json.loads(line)
        v = d.get("version")  # Jackson: an absent / null Long reads as 0
        if v is not None and type(v) is not int:
            raise ValueError(v)
        return {"version": v or 0, "size": d.get("size"), "parts": d.get("parts")}
    except Exception:
        inst = _find_last_complete_checkpoint(log_path)
        return None if inst is None else {"version": inst.version, "size": -1,
                                          "parts": inst.num_parts}


def _find_last_complete_checkpoint(log_path: str) -> Optional[CheckpointInstance]:
    names = sorted(os.listdir(log_path))
    insts = [CheckpointInstance(file_version(n), num_checkpoint_parts(n))
             for n in names if is_checkpoint_file(n)]
    return _latest_complete(insts, None)


def _latest_complete(instances: Sequence[CheckpointInstance],
                     not_later_than: Optional[int]) -> Optional[CheckpointInstance]:
    """getLatestCompleteCheckpointFromList (D/Checkpoints.scala:210-218)."""
    groups: Dict[CheckpointInstance, int] = {}
    for i in instances:
        if not_later_than is None or i.version <= not_later_than:
            groups[i] = groups.get(i, 0) + 1
    complete = [i for i, n in groups.items()
                if (i.num_parts is None and n == 1) or (i.num_parts is not None and n == i.num_parts)]
    if not complete:
        return None
    return max(complete, key=CheckpointInstance.sort_key)


def verify_delta_versions(versions: List[int]) -> None:
    """SnapshotManagement.verifyDeltaVersions (D/SnapshotManagement.scala:365-372)."""
    if versions and list(range(versions[0], versions[-1] + 1)) != versions:
        raise DeltaError("IllegalStateException",
                         "Versions (Vector(%s)) are not contiguous." % ", ".join(map(str, versions)))


def get_log_segment(log_path: str, version_to_load: Optional[int] = None,
                    start_checkpoint: Optional[int] = -1) -> LogSegment:
    """getLogSegmentForVersion (D/SnapshotManagement.scala:82-179). `start_checkpoint=-1`
    means 'use _last_checkpoint' as getSnapshotAtInit does (D/SnapshotManagement.scala:186-206)."""
    if start_checkpoint == -1:
        lc = read_last_checkpoint(log_path)
        start_checkpoint = None if lc is None else lc["version"]
        if version_to_load is not None and start_checkpoint is not None \
                and start_checkpoint > version_to_load:
            start_checkpoint = None
    if not os.path.isdir(log_path):
        raise DeltaError("FileNotFoundException", "No file found in the directory: %s." % log_path)
    start = start_checkpoint or 0
    names = sorted(n for n in os.listdir(log_path))
    new_files = []
    for n in names:
        if not (is_checkpoint_file(n) or is_delta_file(n)):
            continue
        if file_version(n) < start:   # listFrom(prefix of version `start`)
            continue
        if is_checkpoint_file(n) and os.path.getsize(os.path.join(log_path, n)) == 0:
            continue
        if version_to_load is not None and file_version(n) > version_to_load:
            break
        new_files.append(n)
    if not new_files and start_checkpoint is None:
        raise DeltaError("FileNotFoundException", "No file found in the directory: %s." % log_path)
    if not new_files:
        return get_log_segment(log_path, version_to_load, None)
    checkpoints = [n for n in new_files if is_checkpoint_file(n)]
    deltas = [n for n in new_files if is_delta_file(n)]
    insts = [CheckpointInstance(file_version(n), num_checkpoint_parts(n)) for n in checkpoints]
    new_ckpt = _latest_complete(insts, version_to_load)
    if new_ckpt is not None:
        after = [d for d in deltas if file_version(d) > new_ckpt.version]
        vers = [file_version(d) for d in after]
        if vers:
            verify_delta_versions(vers)
            if vers[0] != new_ckpt.version + 1:
                raise DeltaError("IllegalArgumentException",
                                 "requirement failed: Did not get the first delta file version: "
                                 "%d to compute Snapshot" % (new_ckpt.version + 1))
        version = vers[-1] if vers else new_ckpt.version
        return LogSegment(log_path, version, after, new_ckpt.files(), new_ckpt.version)
    if start_checkpoint is not None:
        # DeltaErrors.missingPartFilesException (D/DeltaErrors.scala:543-546)
        raise DeltaError("IllegalStateException",
                         "Couldn't find all part files of the checkpoint version: %d" % start_checkpoint)
    vers = [file_version(d) for d in deltas]
    verify_delta_versions(vers)
    if not vers or vers[0] != 0:
        # DeltaErrors.logFileNotFoundException (D/DeltaErrors.scala:451-457), default retentions
        raise DeltaError("FileNotFoundException", "%s/%s: Unable to reconstruct state at version %s as the "
                         "transaction log has been truncated due to manual deletion or the log retention "
                         "policy (delta.logRetentionDuration=30 days) and checkpoint retention policy "
                         "(delta.checkpointRetentionDuration=2 days)"
                         % (log_path, delta_file(0), vers[-1] if vers else -1))
    return LogSegment(log_path, vers[-1], deltas, [], None)


# ----------------------------------------------------------------------------------------------
# Action model (D/actions/actions.scala:93-542) with Jackson's reading defaults: absent
# primitives read as 0/false, absent Option as None (T/ActionSerializerSuite.scala:94-104).
# ----------------------------------------------------------------------------------------------
ADD, REMOVE, METADATA, TXN, PROTOCOL, CDC, COMMITINFO = (
    "add", "remove", "metaData", "txn", "protocol", "cdc", "commitInfo")
_UNWRAP_ORDER = (ADD, REMOVE, METADATA, TXN, PROTOCOL, CDC, COMMITINFO)  # actions.scala:523-541


def _map_or_none(v):
    if v is None:
        return None
    if isinstance(v, list):  # parquet map -> list of (k, v)
        return {k: val for k, val in v}
    return dict(v)


def make_add(d: dict) -> dict:
    return {
        "path": d.get("path"),
        "partitionValues": _map_or_none(d.get("partitionValues")),
        "size": int(d.get("size") or 0),
        "modificationTime": int(d.get("modificationTime") or 0),
        "dataChange": bool(d.get("dataChange") or False),
        "stats": d.get("stats"),
        "tags": _map_or_none(d.get("tags")),
    }


def make_remove(d: dict) -> dict:
    dt = d.get("deletionTimestamp")
    return {
        "path": d.get("path"),
        "deletionTimestamp": None if dt is None else int(dt),
        "dataChange": bool(d.get("dataChange") or False),
        "extendedFileMetadata": bool(d.get("extendedFileMetadata") or False),
        "partitionValues": _map_or_none(d.get("partitionValues")),
        "size": int(d.get("size") or 0),
        "tags": _map_or_none(d.get("tags")),
    }


def unwrap(single: dict) -> Optional[Tuple[str, dict]]:
    """SingleAction.unwrap priority (D/actions/actions.scala:523-541); unknown-only -> None
    (T/EvolvabilitySuite.scala:43-71)."""
    for k in _UNWRAP_ORDER:
        v = single.get(k)
        if v is not None:
            if k == ADD:
                return ADD, make_add(v)
            if k == REMOVE:
                return REMOVE, make_remove(v)
            return k, v
    return None


def del_timestamp(remove: dict) -> int:  # RemoveFile.delTimestamp (actions.scala:318-319)
    return remove["deletionTimestamp"] if remove["deletionTimestamp"] is not None else 0


# ----------------------------------------------------------------------------------------------
# Path canonicalization (D/Snapshot.scala:301-328) restated for the local-filesystem default:
# an absolute path without scheme/authority is qualified with `file://` (makeQualified on the
# local FS gives scheme `file`, authority ""), everything else is returned as the URI string.
# The replay KEY is java.net.URI equality (D/actions/actions.scala:208-213,
# D/actions/InMemoryLogReplay.scala:40-41); for `file:` URIs an empty authority equals none.
# ----------------------------------------------------------------------------------------------
def _hadoop_normalize(path: str) -> str:
    # Hadoop Path.normalizePath: collapse '//' and drop a trailing '/' (not the root).
    while "//" in path:
        path = path.replace("//", "/")
    if len(path) > 1 and path.endswith("/"):
        path = path[:-1]
    return path


def canonicalize_path(p: str) -> str:
    if p.startswith("/"):
        return "file://" + _hadoop_normalize(p)
    return p


def replay_key(p: str) -> str:
    """URI-equality class of a canonical path string (java.net.URI.equals for file: URIs)."""
    if p.startswith("file:///"):
        return "file:/" + p[len("file:///"):]
    return p


# ----------------------------------------------------------------------------------------------
# Loading the segment's actions in replay order (D/Snapshot.scala:231-263,98-104): checkpoint
# parts first (sorted by file name), then deltas by version; within a file, line/row order.
# ----------------------------------------------------------------------------------------------
def read_json_actions(data: bytes) -> Iterator[Optional[Tuple[str, dict]]]:
    """Spark's JSON reader over Action.logSchema in PERMISSIVE mode (D/DeltaLogFileIndex.scala:67): a
    line that is not a JSON object reads as a row of nulls, which unwrap drops."""
    for line in data.split(b"\n"):
        if not line.strip():
            continue
        try:
            obj = json.loads(line)
        except ValueError:
            yield None
            continue
        yield unwrap(obj) if isinstance(obj, dict) else None


def read_checkpoint_actions(path: str) -> Iterator[Optional[Tuple[str, dict]]]:
    import pyarrow.parquet as pq
    t = pq.read_table(path)
    cols = [c for c in _UNWRAP_ORDER if c in t.column_names]
    for row in t.select(cols).to_pylist():
        yield unwrap(row)


def load_actions(seg: LogSegment) -> Iterator[Tuple[int, Optional[Tuple[str, dict]]]]:
    """Yields (version, action) in the reference's replay order."""
    for name in sorted(seg.checkpoint):
        for a in read_checkpoint_actions(os.path.join(seg.log_path, name)):
            yield seg.checkpoint_version, a
    for name in seg.deltas:
        with open(os.path.join(seg.log_path, name), "rb") as f:
            data = f.read()
        v = file_version(name)
        for a in read_json_actions(data):
            yield v, a


# ----------------------------------------------------------------------------------------------
# InMemoryLogReplay (D/actions/InMemoryLogReplay.scala:35-77)
# ----------------------------------------------------------------------------------------------
class InMemoryLogReplay:
    def __init__(self, min_file_retention_timestamp: int):
        self.min_file_retention_timestamp = min_file_retention_timestamp
        self.current_protocol: Optional[dict] = None
        self.current_version = -1
        self.current_metadata: Optional[dict] = None
        self.transactions: Dict[str, dict] = {}
        self.active_files: Dict[str, dict] = {}   # replay key -> AddFile
        self.tombstones: Dict[str, dict] = {}     # replay key -> RemoveFile

    def append(self, version: int, actions: Iterable[Optional[Tuple[str, dict]]]) -> None:
        assert self.current_version == -1 or version == self.current_version + 1, (
            "Attempted to replay version %d, but state is at %d" % (version, self.current_version))
        self.current_version = version
        for a in actions:
            if a is None:
                continue
            kind, act = a
            if kind == TXN:
                self.transactions[act["appId"]] = act
            elif kind == METADATA:
                self.current_metadata = act
            elif kind == PROTOCOL:
                self.current_protocol = act
            elif kind == ADD:
                add = dict(act, path=canonicalize_path(act["path"]), dataChange=False)
                k = replay_key(add["path"])
                self.active_files[k] = add
                self.tombstones.pop(k, None)
            elif kind == REMOVE:
                rm = dict(act, path=canonicalize_path(act["path"]), dataChange=False)
                k = replay_key(rm["path"])
                self.active_files.pop(k, None)
                self.tombstones[k] = rm
            # commitInfo / cdc: ignored

    def get_tombstones(self) -> List[dict]:
        return [t for t in self.tombstones.values()
                if del_timestamp(t) > self.min_file_retention_timestamp]

    def checkpoint(self) -> List[Tuple[str, dict]]:
        out: List[Tuple[str, dict]] = []
        if self.current_protocol is not None:
            out.append((PROTOCOL, self.current_protocol))
        if self.current_metadata is not None:
            out.append((METADATA, self.current_metadata))
        out.extend((TXN, t) for t in self.transactions.values())
        files = [(ADD, a) for a in self.active_files.values()] + \
                [(REMOVE, r) for r in self.get_tombstones()]
        files.sort(key=lambda kv: kv[1]["path"])
        out.extend(files)
        return out


# ----------------------------------------------------------------------------------------------
# Snapshot (D/Snapshot.scala:88-204)
# ----------------------------------------------------------------------------------------------
@dataclass
class Snapshot:
    version: int
    protocol: Optional[dict]
    metadata: Optional[dict]
    set_transactions: List[dict]
    all_files: List[dict]
    tombstones: List[dict]

    @property
    def size_in_bytes(self) -> int:  # coalesce(sum(add.size), 0)
        return sum(a["size"] for a in self.all_files)

    @property
    def num_of_files(self) -> int:
        return len(self.all_files)

    @property
    def num_of_removes(self) -> int:
        return len(self.tombstones)

    @property
    def num_of_metadata(self) -> int:
        return 0 if self.metadata is None else 1

    @property
    def num_of_protocol(self) -> int:
        return 0 if self.protocol is None else 1

    @property
    def num_of_set_transactions(self) -> int:
        return len(self.set_transactions)

    def counts(self) -> Dict[str, int]:
        return {"numOfFiles": self.num_of_files, "sizeInBytes": self.size_in_bytes,
                "numOfRemoves": self.num_of_removes, "numOfMetadata": self.num_of_metadata,
                "numOfProtocol": self.num_of_protocol,
                "numOfSetTransactions": self.num_of_set_transactions}


def action_not_found(action: str, version: int) -> str:
    """DeltaErrors.actionNotFoundException (D/DeltaErrors.scala:553-560): the stripMargin'd text."""
    return ("\nThe %s of your Delta table couldn't be recovered while Reconstructing\nversion: %d. Did you "
            "manually delete files in the _delta_log directory?\nSet "
            "spark.databricks.delta.stateReconstructionValidation.enabled\nto \"false\" to skip validation.\n"
            "       " % (action, version))


def state_reconstruction(seg: LogSegment, min_file_retention_timestamp: int,
                         validate: bool = True) -> Snapshot:
    """stateReconstruction + computedState. Spark's hash partitioning is a placement detail;
    one reducer over the whole ordered stream computes the same per-key result (each key's
    actions land in one partition, ordered by file)."""
    r = InMemoryLogReplay(min_file_retention_timestamp)
    r.append(0, (a for _, a in load_actions(seg)))
    prot, meta, txns, adds, rms = None, None, [], [], []
    for kind, a in r.checkpoint():
        if kind == PROTOCOL:
            prot = a
        elif kind == METADATA:
            meta = a
        elif kind == TXN:
            txns.append(a)
        elif kind == ADD:
            adds.append(a)
        else:
            rms.append(a)
    if validate and prot is None:  # D/Snapshot.scala:154-162
        raise DeltaError("IllegalStateException", action_not_found("protocol", seg.version))
    if validate and meta is None:  # D/Snapshot.scala:163-171
        raise DeltaError("IllegalStateException", action_not_found("metadata", seg.version))
    return Snapshot(seg.version, prot, meta, txns, adds, rms)


# ----------------------------------------------------------------------------------------------
# Full-record checksum (BASELINE.md "Correctness gate" at sizes where record lists do not fit a
# test): an order-free sum over the survivors of one 64-bit hash per record that covers every field
# the reference's AddFile / RemoveFile carries out of InMemoryLogReplay.checkpoint
# (D/actions/InMemoryLogReplay.scala:55-77; D/actions/actions.scala:220-320; dataChange is forced
# false on both sides, so it is constant). The same definition is computed by the GPU
# (dr_state_record_sums, k_record_hash) and by oracle/replay_oracle.cpp (--record-sums):
#   w0 side (0 add, 1 remove)       w1 xxh64(path, 0)          w2 size
#   w3 add: modificationTime; remove: deletionTimestamp (0 when absent)
#   w4 add: 0; remove: (deletionTimestamp present) | extendedFileMetadata << 1
#   w5 add: xxh64(stats, 1), 0 when null; remove: 0
#   w6 map(partitionValues, 2, 3)   w7 map(tags, 4, 5)
#   map(m, a, b) = 0 when null, else 1 + len(m) + sum over entries of
#                  xxh64(key, a) * 0x9E3779B97F4A7C15 + (0x5BD1E9955BD1E995 if value is null else xxh64(value, b))
#   record = xxh64(w0..w7 as 64 little-endian bytes, 0x5EED);  side sum = sum of records mod 2^64
# ----------------------------------------------------------------------------------------------
_M64 = (1 << 64) - 1
REC_SEED = 0x5EED
_GOLD = 0x9E3779B97F4A7C15
_NULLV = 0x5BD1E9955BD1E995


def _xxh(s: str, seed: int) -> int:
    import xxhash
    return xxhash.xxh64_intdigest(s.encode("utf-8"), seed)


def _map_hash(m: Optional[dict], ks: int, vs: int) -> int:
    if m is None:
        return 0
    h = 1 + len(m)
    for k, v in m.items():
        h += _xxh(k, ks) * _GOLD + (_NULLV if v is None else _xxh(v, vs))
    return h & _M64


def record_hash(rec: dict, side: int) -> int:
    """The canonical hash of one allFiles (side 0) / tombstones (side 1) record (definition above)."""
    import struct
    import xxhash
    if side == 0:
        w3, w4 = rec["modificationTime"], 0
        w5 = 0 if rec.get("stats") is None else _xxh(rec["stats"], 1)
    else:
        dt = rec["deletionTimestamp"]
        w3 = 0 if dt is None else dt
        w4 = (0 if dt is None else 1) | (2 if rec["extendedFileMetadata"] else 0)
        w5 = 0
    w = (side, _xxh(rec["path"], 0), rec["size"] & _M64, w3 & _M64, w4, w5,
         _map_hash(rec.get("partitionValues"), 2, 3), _map_hash(rec.get("tags"), 4, 5))
    return xxhash.xxh64_intdigest(struct.pack("<8Q", *w), REC_SEED)


def record_sums(all_files: Iterable[dict], tombstones: Iterable[dict]) -> Tuple[int, int]:
    """(live_record_sum, tomb_record_sum): order-free full-record checksums of both sides."""
    return (sum(record_hash(r, 0) for r in all_files) & _M64,
            sum(record_hash(r, 1) for r in tombstones) & _M64)


def snapshot_for_table(table_path: str, min_file_retention_timestamp: int,
                       version: Optional[int] = None, validate: bool = True) -> Snapshot:
    seg = get_log_segment(os.path.join(table_path, "_delta_log"), version)
    return state_reconstruction(seg, min_file_retention_timestamp, validate)


# ----------------------------------------------------------------------------------------------
# Partition pruning: DeltaLog.filterFileList / rewritePartitionFilters (D/DeltaLog.scala:500-547)
# with Spark 3.1 non-ANSI Cast(string AS type) and three-valued logic. Predicates are nested
# tuples: ("col", name) ("lit", type, value) ("=",a,b) ("<=>",a,b) ("!=",a,b) ("<",..) ("<=",..)
# (">",..) (">=",..) ("in", a, [lits]) ("isnull", a) ("isnotnull", a) ("and",a,b) ("or",a,b)
# ("not",a). Types: "integer","long","short","byte","date","boolean","string".
# ----------------------------------------------------------------------------------------------
import datetime as _dt

_EPOCH = _dt.date(1970, 1, 1)
_INT_RANGE = {"byte": (-2 ** 7, 2 ** 7 - 1), "short": (-2 ** 15, 2 ** 15 - 1),
              "integer": (-2 ** 31, 2 ** 31 - 1), "long": (-2 ** 63, 2 ** 63 - 1)}
_WS = " \t\n\r\x0b\x0c"


def cast_string(s: Optional[str], typ: str):
    """Cast(UTF8String AS typ), non-ANSI: failure -> None. Canonical forms are pinned; exotic
    forms follow Spark 3.1's UTF8String.toLong/stringToDate as restated here (parity unpinned)."""
    if s is None:
        return None
    if typ == "string":
        return s
    t = s.strip(_WS)
    if typ in _INT_RANGE:
        if not re.fullmatch(r"[+-]?\d+", t):
            return None
        v = int(t)
        lo, hi = _INT_RANGE[typ]
        return v if lo <= v <= hi else None
    if typ == "boolean":
        tl = t.lower()
        if tl in ("t", "true", "y", "yes", "1"):
            return 1
        if tl in ("f", "false", "n", "no", "0"):
            return 0
        return None
    if typ == "date":
        m = re.fullmatch(r"(\d{4})(?:-(\d{1,2})(?:-(\d{1,2})(?:[ T].*)?)?)?", t)
        if not m:
            return None
        y, mo, d = int(m.group(1)), int(m.group(2) or 1), int(m.group(3) or 1)
        try:
            return (_dt.date(y, mo, d) - _EPOCH).days
        except ValueError:
            return None
    return cast_string_v2(s, typ)


# ---- the partitionValues_parsed casts of the other partition types (CheckpointV2.extractPartitionValues,
# D/Checkpoints.scala:380-388: Cast(partitionValues[c] AS type)), restated from Spark 3.1's Cast:
# float / double = Float.parseFloat / Double.parseDouble of the text (Java's FloatingDecimal grammar)
# else Cast.processFloatingPointSpecialLiterals; decimal(p,s) = Decimal.fromString (new
# java.math.BigDecimal(text.trim)) + changePrecision(p, s, ROUND_HALF_UP), null on overflow;
# timestamp = DateTimeUtils.stringToTimestamp in the session zone (UTC here; region zone ids and
# time-only strings are parity unpinned); binary = the UTF-8 bytes. Values: float/double as Python
# floats, decimal as the unscaled int, timestamp as microseconds since the epoch, binary as bytes.
def _java_trim(s: str) -> str:
    return s.strip("".join(chr(c) for c in range(33)))


def cast_string_v2(s: str, typ: str):
    import decimal
    from fractions import Fraction
    t = _java_trim(s)
    if typ in ("float", "double"):
        m = re.fullmatch(r"([+-]?)(?:(NaN)|(Infinity)|((?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)[fFdD]?|"
                         r"0[xX]((?:[0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+))[pP]([+-]?\d+)[fFdD]?)", t)
        if m:
            if m.group(2):
                return float("nan")
            if m.group(3):
                return float("-inf") if m.group(1) == "-" else float("inf")
            if m.group(5) is not None:  # Java's hexadecimal significand with a binary exponent
                h = m.group(5)
                ip, _, fp = h.partition(".")
                x = Fraction(int((ip or "0") + fp, 16), 16 ** len(fp)) * Fraction(2) ** int(m.group(6))
            else:
                x = Fraction(m.group(4))
            if typ == "double":
                v = float(x) if x < Fraction(2) ** 1025 else float("inf")
            else:
                import numpy as np
                # the float32 nearest to the exact value (ties to even), by bracketing with float32
                # neighbours of the double approximation
                fmax = (Fraction(2) - Fraction(1, 1 << 23)) * Fraction(2) ** 127
                if x >= (Fraction(2) - Fraction(1, 1 << 24)) * Fraction(2) ** 127:
                    c = np.float32("inf")
                else:
                    c = np.float32(float(min(x, fmax)))
                if np.isfinite(c):
                    with np.errstate(over="ignore"):
                        cand = [np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))]
                    cand = [k for k in cand if np.isfinite(k)]
                    c = min(cand, key=lambda k: (abs(Fraction(float(k)) - x), int(np.float32(k).view(np.uint32)) & 1))
                v = float(c)
            return -v if m.group(1) == "-" else v
        tl = t.lower()
        if tl in ("inf", "+inf", "infinity", "+infinity"):
            return float("inf")
        if tl in ("-inf", "-infinity"):
            return float("-inf")
        return float("nan") if tl == "nan" else None
    if typ == "binary":
        return s.encode("utf-8")
    if typ == "timestamp":
        m = re.fullmatch(r"([+-]?)(\d{4,6})(?:-(\d{1,2})(?:-(\d{1,2})(?:[ T](\d{1,2}):(\d{1,2})"
                         r"(?::(\d{1,2})(?:\.(\d*))?)?(.*))?)?)?", t)
        if not m:
            return None
        sign, y, mo, d, hh, mi, ss, frac, zone = m.groups()
        try:
            day = (_dt.date(int(y) * (-1 if sign == "-" else 1), int(mo or 1), int(d or 1)) - _EPOCH).days
        except ValueError:
            return None
        hh, mi, ss = int(hh or 0), int(mi or 0), int(ss or 0)
        if hh > 23 or mi > 59 or ss > 59:
            return None
        off = 0
        if zone:
            z = re.fullmatch(r"Z|(?:UTC|GMT|UT)?(?:([+-])(\d{1,2})(?::?(\d{1,2})(?::?(\d{1,2}))?)?)?", _java_trim(zone))
            if not z or not zone.strip():
                return None
            if z.group(1):
                h, mn, sc = int(z.group(2)), int(z.group(3) or 0), int(z.group(4) or 0)
                if h > 18 or mn > 59 or sc > 59:
                    return None
                off = (h * 3600 + mn * 60 + sc) * (-1 if z.group(1) == "-" else 1)
        return ((day * 86400 + hh * 3600 + mi * 60 + ss) - off) * 1_000_000 + int(((frac or "") + "000000")[:6])
    m = re.fullmatch(r"decimal(?:\((\d+),(\d+)\))?", typ)
    if m:
        p, sc = (int(m.group(1)), int(m.group(2))) if m.group(1) else (10, 0)
        if not re.fullmatch(r"[+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?", t):
            return None
        q = Fraction(decimal.Decimal(t)) * 10 ** sc
        mag = abs(q)
        unscaled = int(mag) + (1 if mag - int(mag) >= Fraction(1, 2) else 0)  # ROUND_HALF_UP
        if unscaled >= 10 ** p:
            return None
        return -unscaled if q < 0 else unscaled
    raise ValueError("unsupported partition type %s" % typ)


def _cmp(op, a, b):
    if a is None or b is None:
        return None
    return {"=": a == b, "!=": a != b, "<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]


def _lit_value(typ: str, v):
    if v is None:
        return None
    if typ == "date" and isinstance(v, str):
        return cast_string(v, "date")
    if typ == "boolean":
        return 1 if v else 0
    return v


def eval_predicate(expr, pv: Dict[str, Optional[str]], schema: Dict[str, str]):
    op = expr[0]
    if op == "col":
        # rewritePartitionFilters (D/DeltaLog.scala:525-546): backticks stripped, the partition
        # field found with the (case-insensitive) resolver, Cast(partitionValues[field] AS type);
        # an unknown column stays an uncast map lookup
        name = expr[1].strip("`")
        field = next((f for f in schema if f.lower() == name.lower()), None)
        if field is None:
            return (pv or {}).get(name)
        return cast_string((pv or {}).get(field), schema[field])
    if op == "lit":
        return _lit_value(expr[1], expr[2])
    if op in ("=", "!=", "<", "<=", ">", ">="):
        return _cmp(op, eval_predicate(expr[1], pv, schema), eval_predicate(expr[2], pv, schema))
    if op == "<=>":
        a, b = eval_predicate(expr[1], pv, schema), eval_predicate(expr[2], pv, schema)
        return (a is None and b is None) or (a is not None and b is not None and a == b)
    if op == "in":
        a = eval_predicate(expr[1], pv, schema)
        if a is None:
            return None
        vals = [eval_predicate(l, pv, schema) for l in expr[2]]
        if any(v == a for v in vals if v is not None):
            return True
        return None if any(v is None for v in vals) else False
    if op == "isnull":
        return eval_predicate(expr[1], pv, schema) is None
    if op == "isnotnull":
        return eval_predicate(expr[1], pv, schema) is not None
    if op == "and":
        a, b = eval_predicate(expr[1], pv, schema), eval_predicate(expr[2], pv, schema)
        if a is False or b is False:
            return False
        return None if (a is None or b is None) else True
    if op == "or":
        a, b = eval_predicate(expr[1], pv, schema), eval_predicate(expr[2], pv, schema)
        if a is True or b is True:
            return True
        return None if (a is None or b is None) else False
    if op == "not":
        a = eval_predicate(expr[1], pv, schema)
        return None if a is None else (not a)
    raise ValueError(op)


def partition_schema(metadata: dict) -> Dict[str, str]:
    """Metadata.partitionSchema (D/actions/actions.scala:370-373)."""
    schema = json.loads(metadata["schemaString"])
    fields = {f["name"]: f["type"] for f in schema["fields"]}
    return {c: fields[c] for c in metadata.get("partitionColumns") or []}


def filter_file_list(schema: Dict[str, str], files: List[dict], filters: Sequence) -> List[dict]:
    """filterFileList: AND of the rewritten filters, keep rows where it is TRUE."""
    out = []
    for f in files:
        ok = True
        for e in filters:
            if eval_predicate(e, f["partitionValues"], schema) is not True:
                ok = False
                break
        if ok:
            out.append(f)
    return out


def crc_counts(log_path: str, version: int) -> Optional[dict]:
    """The `.crc` VersionChecksum (D/Checksum.scala:45-192) if present."""
    p = os.path.join(log_path, "%020d.crc" % version)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.loads(f.readline())
