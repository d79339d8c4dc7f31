"""Checkpoint writer from the resident state (rows a20 / a21).

`Checkpoints.writeCheckpoint` / `buildCheckpoint` (D/Checkpoints.scala:229-365) writes the
snapshot's state -- protocol, metaData, txns, live AddFiles and unexpired RemoveFiles, commitInfo
and cdc dropped, every record with dataChange=false -- as one Parquet file of SingleAction rows,
checks that it holds numOfFiles adds, and records `_last_checkpoint` = {"version", "size"}. The
`add` struct is rebuilt as (path, partitionValues, size, modificationTime, dataChange, tags), then
`stats` while the table property `delta.checkpoint.writeStatsAsJson` holds (default true,
D/DeltaConfig.scala:401-406), then `partitionValues_parsed` -- every partition column of the
metadata's partition schema cast to its type (CheckpointV2.extractPartitionValues, :372-389) --
when `delta.checkpoint.writeStatsAsStruct` is true or, unset, `checkpointV2.enabled` is (default
true, D/sources/DeltaSQLConf.scala:363-368) and the table is partitioned. The schema is nullable
throughout (`chk.schema.asNullable`).

Here the records come from the GPU state through `dr_state_export`'s columnar buffers (gathered
on the device) and are turned into Arrow columns without per-record Python objects; Arrow's
Parquet C++ writer encodes them (SNAPPY, dictionary pages). `parts > 1` writes the protocol's
multi-part form (FileNames.checkpointFileWithParts, D/util/FileNames.scala:70-73; PROTOCOL.md
"Checkpoints"): part i of n holds a contiguous slice of the rows and `_last_checkpoint` carries
"parts". A sharded replay's ranks each hold a path-hash shard of the state and can write their own
part with `write_part` (rank 0 then writes `_last_checkpoint`).
"""
import ctypes as C
import json
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N


def _np(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,)).copy()


def _bytes(ptr, n):
    return C.string_at(ptr, n) if n else b""


def _strings(pa, off_ptr, data_ptr, n, null=None):
    off = _np(off_ptr, n + 1, np.int64)
    data = _bytes(data_ptr, int(off[-1]) if n else 0)
    mask = None if null is None else pa.py_buffer(np.packbits(~null.astype(bool), bitorder="little").tobytes())
    return pa.LargeStringArray.from_buffers(n, pa.py_buffer(off.tobytes()), pa.py_buffer(data), mask,
                                            int(null.sum()) if null is not None else 0).cast(pa.string())


def _map(pa, e, pre, n):
    entry_off = _np(getattr(e, pre + "_entry_off"), n + 1, np.int64)
    m = int(entry_off[-1]) if n else 0
    keys = _strings(pa, getattr(e, pre + "_key_off"), getattr(e, pre + "_key_bytes"), m)
    vnull = _np(getattr(e, pre + "_val_null"), m, np.uint8)
    vals = _strings(pa, getattr(e, pre + "_val_off"), getattr(e, pre + "_val_bytes"), m, vnull)
    null = _np(getattr(e, pre + "_null"), n, np.uint8).astype(bool)
    offs = pa.array(entry_off.astype(np.int32), pa.int32())
    return pa.MapArray.from_arrays(offs, keys, vals, mask=pa.array(null) if null.any() else None)


_PARSED_TYPES = {"string": "string", "byte": "int8", "short": "int16", "integer": "int32", "long": "int64",
                 "date": "date32", "boolean": "bool_", "float": "float32", "double": "float64", "binary": "binary"}


def _parsed_type(pa, t: str):
    """Arrow type of a partition column in partitionValues_parsed (the Spark type's Parquet layout)."""
    import re
    if t in _PARSED_TYPES:
        return getattr(pa, _PARSED_TYPES[t])()
    if t == "timestamp":
        return pa.timestamp("us", tz="UTC")  # written as INT96, Spark's outputTimestampType default
    m = re.fullmatch(r"decimal(?:\((\d+),(\d+)\))?", t)
    if m:
        return pa.decimal128(int(m.group(1)), int(m.group(2))) if m.group(1) else pa.decimal128(10, 0)
    raise KeyError(t)


def _conf_bool(md, key: str, default):
    v = ((md or {}).get("configuration") or {}).get(key)
    return default if v is None else str(v).strip().lower() == "true"


def checkpoint_options(md, checkpoint_v2_enabled: bool = True):
    """(write stats as JSON, partition schema of partitionValues_parsed or None) from the metadata
    (D/Checkpoints.scala:340-352)."""
    from .predicates import partition_schema
    stats = _conf_bool(md, "delta.checkpoint.writeStatsAsJson", True)
    struct = _conf_bool(md, "delta.checkpoint.writeStatsAsStruct", None)
    if struct is None:
        struct = checkpoint_v2_enabled
    schema = partition_schema(md) if md else {}
    return stats, (schema if struct and schema else None)


def _types(pa, stats=True, parsed=None):
    mt = pa.map_(pa.string(), pa.string())
    add_f = [("path", pa.string()), ("partitionValues", mt), ("size", pa.int64()),
             ("modificationTime", pa.int64()), ("dataChange", pa.bool_()), ("tags", mt)]
    if stats:
        add_f.append(("stats", pa.string()))
    if parsed:
        add_f.append(("partitionValues_parsed",
                      pa.struct([(c, _parsed_type(pa, t)) for c, t in parsed.items()])))
    add_t = pa.struct(add_f)
    rm_t = pa.struct([("path", pa.string()), ("deletionTimestamp", pa.int64()), ("dataChange", pa.bool_()),
                      ("extendedFileMetadata", pa.bool_()), ("partitionValues", mt), ("size", pa.int64()),
                      ("tags", mt)])
    txn_t = pa.struct([("appId", pa.string()), ("version", pa.int64()), ("lastUpdated", pa.int64())])
    fmt_t = pa.struct([("provider", pa.string()), ("options", mt)])
    md_t = pa.struct([("id", pa.string()), ("name", pa.string()), ("description", pa.string()),
                      ("format", fmt_t), ("schemaString", pa.string()),
                      ("partitionColumns", pa.list_(pa.string())), ("configuration", mt),
                      ("createdTime", pa.int64())])
    prot_t = pa.struct([("minReaderVersion", pa.int32()), ("minWriterVersion", pa.int32())])
    return mt, add_t, rm_t, txn_t, md_t, prot_t


def _parsed_struct(pa, pv, parsed, typ):
    """Cast(add.partitionValues[c] AS type) per partition column: a missing key or a failed
    non-ANSI cast is null (the device filter's cast grammar, predicates.cast_partition_value)."""
    from .predicates import cast_partition_value
    keys = pv.keys.to_pylist() if len(pv) else []
    items = pv.items.to_pylist() if len(pv) else []
    offs = pv.offsets.to_pylist() if len(pv) else [0]
    nulls = pv.is_null().to_pylist() if len(pv) else []
    cols = {c: [] for c in parsed}
    for i in range(len(pv)):
        m = {} if nulls[i] else {keys[j]: items[j] for j in range(offs[i], offs[i + 1])}
        for c, t in parsed.items():
            cols[c].append(cast_partition_value(m.get(c), t))
    arrays = [pa.array(cols[c], f.type) for c, f in zip(parsed, typ)]
    return pa.StructArray.from_arrays(arrays, fields=list(typ))


def _file_struct(pa, state, which, typ, stats=True, parsed=None):
    e = N.dr_export()
    state.eng.check(state.eng.lib.dr_state_export(state.h, which, C.byref(e)))
    n = int(e.n)
    path = _strings(pa, e.path_off, e.path_bytes, n)
    pv = _map(pa, e, "pv", n)
    tags = _map(pa, e, "tags", n)
    size = pa.array(_np(e.size, n, np.int64), pa.int64())
    dc = pa.array(np.zeros(n, bool), pa.bool_())
    if which == N.DR_LIVE:
        cols = [path, pv, size, pa.array(_np(e.modification_time, n, np.int64), pa.int64()), dc, tags]
        if stats:
            cols.append(_strings(pa, e.stats_off, e.stats_bytes, n, _np(e.stats_null, n, np.uint8)))
        if parsed:
            cols.append(_parsed_struct(pa, pv, parsed, typ.field("partitionValues_parsed").type))
    else:
        valid = _np(e.deletion_timestamp_valid, n, np.uint8).astype(bool)
        dts = pa.array(_np(e.deletion_timestamp, n, np.int64), pa.int64(), mask=~valid)
        efm = pa.array(_np(e.extended_file_metadata, n, np.uint8).astype(bool), pa.bool_())
        cols = [path, dts, dc, efm, pv, size, tags]
    return pa.StructArray.from_arrays(cols, fields=list(typ)), n


def _nonfile_rows(state):
    prot, md, txns = None, None, []
    for a in state.nonfile:
        if "protocol" in a:
            prot = a["protocol"]
        elif "metaData" in a:
            md = a["metaData"]
        elif "txn" in a:
            txns.append(a["txn"])
    return prot, md, txns


def checkpoint_table(state, checkpoint_v2_enabled: bool = True):
    """The checkpoint rows of a GPU state as an Arrow table (protocol, metaData, txns, adds,
    removes; columns txn, add, remove, metaData, protocol)."""
    import pyarrow as pa
    prot, md, txns = _nonfile_rows(state)
    stats, parsed = checkpoint_options(md, checkpoint_v2_enabled)
    mt, add_t, rm_t, txn_t, md_t, prot_t = _types(pa, stats, parsed)
    adds, na = _file_struct(pa, state, N.DR_LIVE, add_t, stats, parsed)
    rms, nr = _file_struct(pa, state, N.DR_TOMBSTONES, rm_t)
    head = []
    if prot is not None:
        head.append({"protocol": {"minReaderVersion": prot.get("minReaderVersion", 0),
                                  "minWriterVersion": prot.get("minWriterVersion", 0)}})
    if md is not None:
        fmt = md.get("format") or {}
        head.append({"metaData": {
            "id": md.get("id"), "name": md.get("name"), "description": md.get("description"),
            "format": {"provider": fmt.get("provider"), "options": list((fmt.get("options") or {}).items())},
            "schemaString": md.get("schemaString"), "partitionColumns": md.get("partitionColumns"),
            "configuration": list((md.get("configuration") or {}).items()), "createdTime": md.get("createdTime")}})
    for t in txns:
        head.append({"txn": {"appId": t.get("appId"), "version": t.get("version", 0),
                             "lastUpdated": t.get("lastUpdated")}})
    h = len(head)

    def col(name, typ):
        return pa.array([r.get(name) for r in head], typ)

    def cat(head_arr, body, typ, at):
        parts = [head_arr]
        for k, (arr, n) in enumerate(body):
            parts.append(arr if k == at else pa.nulls(n, typ))
        return pa.concat_arrays([p for p in parts if len(p)]) if h + na + nr else pa.array([], typ)

    body = [(adds, na), (rms, nr)]
    table = pa.Table.from_arrays([
        cat(col("txn", txn_t), body, txn_t, -1),
        cat(pa.nulls(h, add_t), body, add_t, 0),
        cat(pa.nulls(h, rm_t), body, rm_t, 1),
        cat(col("metaData", md_t), body, md_t, -1),
        cat(col("protocol", prot_t), body, prot_t, -1),
    ], names=["txn", "add", "remove", "metaData", "protocol"])
    return table, na


def check_add_rows(written: int, num_of_files: int) -> None:
    """Checkpoints.writeCheckpoint's check before `_last_checkpoint` is written: the add rows the parts
    hold must be the snapshot's numOfFiles (D/Checkpoints.scala:325-328)."""
    if written != num_of_files:
        from .delta_log import DeltaError
        raise DeltaError(15, "State of the checkpoint doesn't match that of the snapshot.")


def checkpoint_file_with_parts(log_path: str, version: int, part: int, parts: int) -> str:
    return os.path.join(log_path, "%020d.checkpoint.%010d.%010d.parquet" % (version, part, parts))


def write_part(state, log_path: str, version: int, part: int, parts: int, row_group_size: int = 1 << 20) -> int:
    """One part (1-based) of a multi-part checkpoint from one shard's state; returns its row count."""
    import pyarrow.parquet as pq
    table, _ = checkpoint_table(state)
    path = checkpoint_file_with_parts(log_path, version, part, parts)
    tmp = os.path.join(os.path.dirname(path), ".%s.tmp" % os.path.basename(path))
    pq.write_table(table, tmp, compression="snappy", row_group_size=row_group_size, write_statistics=False,
                   use_deprecated_int96_timestamps=True, store_decimal_as_integer=True)
    os.replace(tmp, path)
    return table.num_rows


def write_checkpoint_device(snapshot, parts: int = 1, row_group_size: int = 1 << 20,
                            checkpoint_v2_enabled: bool = True) -> dict:
    """writeCheckpoint with the Parquet pages of the file actions encoded on the GPU
    (dr_state_write_checkpoint); same files and `_last_checkpoint` as `write_checkpoint`."""
    state = snapshot.state
    md = next((a["metaData"] for a in state.nonfile if "metaData" in a), None)
    stats, parsed = checkpoint_options(md, checkpoint_v2_enabled)
    log_path = snapshot.delta_log.log_path
    rows = adds = 0
    for i in range(parts):
        data, n, na = state.write_checkpoint_part(i + 1, parts, stats=stats, parsed=parsed is not None,
                                                  row_group_rows=row_group_size, with_adds=True)
        rows += n
        adds += na
        path = (os.path.join(log_path, "%020d.checkpoint.parquet" % snapshot.version) if parts <= 1
                else checkpoint_file_with_parts(log_path, snapshot.version, i + 1, parts))
        tmp = os.path.join(os.path.dirname(path), ".%s.tmp" % os.path.basename(path))
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    check_add_rows(adds, snapshot.num_of_files)
    meta = {"version": snapshot.version, "size": rows}
    if parts > 1:
        meta["parts"] = parts
    write_last_checkpoint(log_path, meta)
    return meta


def write_checkpoint(snapshot, parts: int = 1, row_group_size: int = 1 << 20) -> dict:
    """writeCheckpoint for a GPU snapshot: the checkpoint file(s) of snapshot.version and
    `_last_checkpoint`; returns the CheckpointMetaData written there."""
    import pyarrow.parquet as pq
    table, n_adds = checkpoint_table(snapshot.state)
    check_add_rows(n_adds, snapshot.num_of_files)  # D/Checkpoints.scala:325-328
    log_path = snapshot.delta_log.log_path
    rows = table.num_rows
    if parts <= 1:
        paths = [os.path.join(log_path, "%020d.checkpoint.parquet" % snapshot.version)]
        slices = [table]
    else:
        paths = [checkpoint_file_with_parts(log_path, snapshot.version, i + 1, parts) for i in range(parts)]
        step = (rows + parts - 1) // parts
        slices = [table.slice(i * step, max(0, min(step, rows - i * step))) for i in range(parts)]
    for path, t in zip(paths, slices):
        tmp = os.path.join(os.path.dirname(path), ".%s.tmp" % os.path.basename(path))
        # decimals as Spark's non-legacy layout: INT32 up to precision 9, INT64 up to 18 (the device
        # writer's), FIXED_LEN_BYTE_ARRAY beyond
        pq.write_table(t, tmp, compression="snappy", row_group_size=row_group_size, write_statistics=False,
                       use_deprecated_int96_timestamps=True, store_decimal_as_integer=True)
        os.replace(tmp, path)  # a reader never sees a partial part
    meta = {"version": snapshot.version, "size": rows}
    if parts > 1:
        meta["parts"] = parts
    write_last_checkpoint(log_path, meta)
    return meta


def write_last_checkpoint(log_path: str, meta: dict) -> None:
    """`_last_checkpoint` through a temp file + rename, so a concurrent reader sees the old or the
    new file whole (a partial file would be taken as corrupted, D/Checkpoints.scala:166-173)."""
    tmp = os.path.join(log_path, "._last_checkpoint.%d.tmp" % os.getpid())
    with open(tmp, "w") as f:
        f.write(json.dumps(meta, separators=(",", ":")) + "\n")
    os.replace(tmp, os.path.join(log_path, "_last_checkpoint"))
