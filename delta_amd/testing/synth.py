"""Seeded synthetic `_delta_log` generator for the BASELINE.json configs.

Writes newline-delimited JSON commits in the field order Jackson produces for the reference's
case classes (D/actions/actions.scala:220-320; D/util/JsonUtils.scala:26-31) and Parquet
checkpoints with the checkpoint column layout of D/Checkpoints.scala:340-389 (v1 data pages,
dictionary encoding, SNAPPY) written by pyarrow. All text is built with vectorised pyarrow
compute kernels, so a 10M-file table is generated in well under a minute.

Every table also gets its expected result *by construction* (which file ids are live, which
tombstones survive the cutoff, the aggregate counts): a size-independent check that does not
need any replay at all.

File identity: file id `i` has path
  p0=<date>/p1=<int>[/p2=<word>/p3=<bool>]/part-<5 digits>-<uuid>-c000.snappy.parquet
(~88 bytes, URI-safe, relative).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

BASE_SEED = 0xDE17A
T0 = 1_700_000_000_000  # modificationTime base (ms)
DAY_MS = 86_400_000
WORDS = ["w%d" % i for i in range(64)]
PART_COLS = ["p0", "p1", "p2", "p3"]
PART_TYPES = {"p0": "date", "p1": "integer", "p2": "string", "p3": "boolean"}
HIVE_NULL = "__HIVE_DEFAULT_PARTITION__"
_DATES = [str(np.datetime64("2020-01-01") + np.timedelta64(d, "D")) for d in range(365)]


def _pa():
    import pyarrow as pa
    import pyarrow.compute as pc
    return pa, pc


@dataclass
class Expected:
    version: int
    min_file_retention_timestamp: int
    num_files: int
    size_in_bytes: int
    num_removes: int
    num_actions: int           # SURVEY §8d unit of work: non-blank JSON lines + checkpoint rows
    num_file_actions: int
    live_ids: Optional[np.ndarray] = None
    tomb_ids: Optional[np.ndarray] = None
    json_bytes: int = 0
    checkpoint_bytes: int = 0


class FilePool:
    """Vectorised description of every file id the generator mints."""

    def __init__(self, rng: np.random.Generator, n: int, ncols: int):
        self.ncols = ncols
        self.p0 = rng.integers(0, 365, n, dtype=np.int32)             # days after 2020-01-01
        self.p1 = rng.integers(0, 1000, n, dtype=np.int32)
        self.p2 = rng.integers(0, 64, n, dtype=np.int32)
        self.p2null = rng.random(n) < 0.01
        self.p3 = rng.integers(0, 2, n, dtype=np.int8)
        self.part = rng.integers(0, 100000, n, dtype=np.int32)
        self.uuid = rng.integers(0, 2 ** 63, (n, 2), dtype=np.int64)
        self.size = np.exp(rng.uniform(np.log(1024), np.log(256 * 2 ** 20), n)).astype(np.int64)
        self.nrec = rng.integers(1, 1_000_000, n, dtype=np.int64)
        self.minv = rng.integers(0, 1000, n, dtype=np.int64)

    def __len__(self):
        return len(self.p0)

    # -- vectorised string columns for an id array ---------------------------------------------
    def _uuid(self, ids):
        pa, _ = _pa()
        n = len(ids)
        u = self.uuid[ids]
        b = np.concatenate([u[:, 0].astype(">u8").view(np.uint8).reshape(n, 8),
                            u[:, 1].astype(">u8").view(np.uint8).reshape(n, 8)], axis=1)
        hexd = np.frombuffer(b"0123456789abcdef", np.uint8)
        nib = np.empty((n, 32), np.uint8)
        nib[:, 0::2] = hexd[b >> 4]
        nib[:, 1::2] = hexd[b & 15]
        out = np.full((n, 36), ord("-"), np.uint8)
        out[:, 0:8], out[:, 9:13], out[:, 14:18] = nib[:, 0:8], nib[:, 8:12], nib[:, 12:16]
        out[:, 19:23], out[:, 24:36] = nib[:, 16:20], nib[:, 20:32]
        return pa.array(out.view("S36").ravel() if n else np.zeros(0, "S36")).cast(pa.string())

    def date_s(self, ids):
        pa, _ = _pa()
        return pa.array(_DATES, pa.string()).take(pa.array(self.p0[ids]))

    def p1_s(self, ids):
        pa, pc = _pa()
        return pc.cast(pa.array(self.p1[ids]), pa.string())

    def p2_s(self, ids, null_token):
        pa, _ = _pa()
        words = pa.array(WORDS + [null_token], pa.string())
        return words.take(pa.array(np.where(self.p2null[ids], 64, self.p2[ids])))

    def p3_s(self, ids):
        pa, _ = _pa()
        return pa.array(["false", "true"], pa.string()).take(pa.array(self.p3[ids].astype(np.int64)))

    def paths(self, ids):
        pa, pc = _pa()
        parts = ["p0=", self.date_s(ids), "/p1=", self.p1_s(ids)]
        if self.ncols >= 4:
            parts += ["/p2=", self.p2_s(ids, HIVE_NULL), "/p3=", self.p3_s(ids)]
        parts += ["/part-", pc.utf8_lpad(pc.cast(pa.array(self.part[ids]), pa.string()), 5, "0"), "-",
                  self._uuid(ids), "-c000.snappy.parquet"]
        return pc.binary_join_element_wise(*parts, "")

    def stats(self, ids, escaped=False):
        pa, pc = _pa()
        q = '\\"' if escaped else '"'
        nr, mv = self.nrec[ids], self.minv[ids]
        s = lambda a: pc.cast(pa.array(a), pa.string())
        return pc.binary_join_element_wise(
            "{%snumRecords%s:" % (q, q), s(nr), ",%sminValues%s:{%sid%s:" % (q, q, q, q), s(mv),
            "},%smaxValues%s:{%sid%s:" % (q, q, q, q), s(mv + nr),
            "},%snullCount%s:{%sid%s:0}}" % (q, q, q, q), "")

    def pv_json(self, ids):
        pa, pc = _pa()
        parts = ['{"p0":"', self.date_s(ids), '","p1":"', self.p1_s(ids), '"']
        if self.ncols >= 4:
            p2 = self.p2_s(ids, "\x00")
            quoted = pc.binary_join_element_wise('"', p2, '"', "")
            p2j = pc.if_else(pc.equal(p2, "\x00"), "null", quoted)
            parts += [',"p2":', p2j, ',"p3":"', self.p3_s(ids), '"']
        parts.append("}")
        return pc.binary_join_element_wise(*parts, "")

    # scalar helpers (tests, edge corpora)
    def path(self, i) -> str:
        return self.paths(np.array([i]))[0].as_py()

    def pvals(self, i):
        d = {"p0": _DATES[self.p0[i]], "p1": str(int(self.p1[i]))}
        if self.ncols >= 4:
            d["p2"] = None if self.p2null[i] else WORDS[self.p2[i]]
            d["p3"] = "true" if self.p3[i] else "false"
        return d


def _flat(x):
    pa, _ = _pa()
    return x.combine_chunks() if isinstance(x, pa.ChunkedArray) else x


def _i64s(a):
    pa, pc = _pa()
    return pc.cast(pa.array(np.asarray(a, dtype=np.int64)), pa.string())


def add_lines(pool: FilePool, ids, mtimes):
    _, pc = _pa()
    return pc.binary_join_element_wise(
        '{"add":{"path":"', pool.paths(ids), '","partitionValues":', pool.pv_json(ids), ',"size":',
        _i64s(pool.size[ids]), ',"modificationTime":', _i64s(mtimes), ',"dataChange":true,"stats":"',
        pool.stats(ids, escaped=True), '"}}\n', "")


def remove_lines(pool: FilePool, ids, del_ts):
    _, pc = _pa()
    return pc.binary_join_element_wise(
        '{"remove":{"path":"', pool.paths(ids), '","deletionTimestamp":', _i64s(del_ts),
        ',"dataChange":true,"extendedFileMetadata":true,"partitionValues":', pool.pv_json(ids),
        ',"size":', _i64s(pool.size[ids]), '}}\n', "")


def _text_bytes(arr) -> bytes:
    """Concatenated bytes of a string array (each element already ends with a newline)."""
    arr = _flat(arr)
    if len(arr) == 0:
        return b""
    off = np.frombuffer(arr.buffers()[1], dtype=np.int32, count=len(arr) + 1, offset=arr.offset * 4)
    data = arr.buffers()[2]
    return data.to_pybytes()[off[0]:off[-1]]


def add_line(pool: FilePool, i: int, mtime: int) -> str:
    return add_lines(pool, np.array([i]), np.array([mtime]))[0].as_py().rstrip("\n")


def remove_line(pool: FilePool, i: int, del_ts: int) -> str:
    return remove_lines(pool, np.array([i]), np.array([del_ts]))[0].as_py().rstrip("\n")


def protocol_line() -> str:
    return '{"protocol":{"minReaderVersion":1,"minWriterVersion":2}}'


def schema_string(ncols: int) -> str:
    fields = [{"name": "id", "type": "long", "nullable": True, "metadata": {}}]
    for c in PART_COLS[:ncols]:
        fields.append({"name": c, "type": PART_TYPES[c], "nullable": True, "metadata": {}})
    return json.dumps({"type": "struct", "fields": fields}, separators=(",", ":"))


def metadata_dict(ncols: int, configuration: Optional[dict] = None) -> dict:
    return {"id": "00000000-0000-4000-8000-00000000de17", "format": {"provider": "parquet", "options": {}},
            "schemaString": schema_string(ncols), "partitionColumns": PART_COLS[:ncols],
            "configuration": configuration or {}, "createdTime": T0}


def metadata_line(ncols: int) -> str:
    return json.dumps({"metaData": metadata_dict(ncols)}, separators=(",", ":"))


def commit_info_line(version: int, op: str = "WRITE") -> str:
    return ('{"commitInfo":{"timestamp":%d,"operation":"%s","operationParameters":{"mode":"Append",'
            '"partitionBy":"[]"},"readVersion":%d,"isBlindAppend":false}}'
            % (T0 + version * 60000, op, max(version - 1, 0)))


def delta_name(v: int) -> str:
    return "%020d.json" % v


# ----------------------------------------------------------------------------------------------
# Checkpoint writer (pyarrow) -- exact checkpoint layout (D/Checkpoints.scala:354-389)
# ----------------------------------------------------------------------------------------------
def write_checkpoint(path: str, pool: FilePool, add_ids: np.ndarray, ncols: int, version: int,
                     with_parsed: bool = False, row_group_size: int = 1 << 20,
                     data_page_size: int = 1 << 20, compression: str = "snappy",
                     data_page_version: str = "1.0", use_dictionary: bool = True, head: bool = True) -> int:
    """Rows: protocol, metaData (unless `head` is false: later parts of a multi-part checkpoint),
    then one `add` per id. Returns the row count."""
    pa, pc = _pa()
    import pyarrow.parquet as pq

    n = len(add_ids)
    h = 2 if head else 0
    nrows = n + h
    mt = pa.map_(pa.string(), pa.string())
    add_valid = np.concatenate([np.zeros(h, bool), np.ones(n, bool)])
    null2 = pa.nulls(h, pa.string())
    paths = pa.concat_arrays([null2, _flat(pool.paths(add_ids))])
    stats = pa.concat_arrays([null2, _flat(pool.stats(add_ids))])
    # partitionValues map: keys/items interleaved per row
    cols = PART_COLS[:ncols]
    vals = [pool.date_s(add_ids), pool.p1_s(add_ids)]
    if ncols >= 4:
        vals += [pc.if_else(pa.array(pool.p2null[add_ids]), pa.scalar(None, pa.string()),
                            pool.p2_s(add_ids, "")), pool.p3_s(add_ids)]
    allv = pa.concat_arrays([_flat(v) for v in vals])
    inter = (np.arange(n)[:, None] + np.arange(ncols)[None, :] * n).ravel()
    items = allv.take(pa.array(inter))
    keys = pa.array(np.tile(np.array(cols, dtype=object), n), pa.string())
    offs = np.concatenate([np.zeros(h, np.int64), np.arange(n + 1) * ncols]).astype(np.int32)
    pv_arr = pa.MapArray.from_arrays(pa.array(offs), keys, items)
    zeros2 = np.zeros(h, np.int64)
    add_fields = [
        paths, pv_arr,
        pa.array(np.concatenate([zeros2, pool.size[add_ids]]), pa.int64()),
        pa.array(np.concatenate([zeros2, T0 + version * 60000 + np.arange(n, dtype=np.int64) % 60000]),
                 pa.int64()),
        pa.array(np.zeros(nrows, bool)),
        pa.nulls(nrows, mt),
        stats,
    ]
    add_names = ["path", "partitionValues", "size", "modificationTime", "dataChange", "tags", "stats"]
    add_types = [pa.string(), mt, pa.int64(), pa.int64(), pa.bool_(), mt, pa.string()]
    if with_parsed and ncols:
        parsed_arrays, parsed_fields = [], []
        for c in cols:
            if c == "p0":
                arr = pa.array(np.concatenate([zeros2, pool.p0[add_ids] + 18262]).astype(np.int32), pa.date32())
            elif c == "p1":
                arr = pa.array(np.concatenate([zeros2, pool.p1[add_ids]]).astype(np.int32), pa.int32())
            elif c == "p2":
                arr = pa.concat_arrays([null2, _flat(pc.if_else(pa.array(pool.p2null[add_ids]),
                                                                pa.scalar(None, pa.string()), pool.p2_s(add_ids, "")))])
            else:
                arr = pa.array(np.concatenate([zeros2, pool.p3[add_ids]]).astype(bool), pa.bool_())
            parsed_arrays.append(arr)
            parsed_fields.append(pa.field(c, arr.type))
        add_fields.append(pa.StructArray.from_arrays(parsed_arrays, fields=parsed_fields))
        add_names.append("partitionValues_parsed")
        add_types.append(pa.struct(parsed_fields))
    add_struct = pa.StructArray.from_arrays(
        add_fields, fields=[pa.field(nm, t) for nm, t in zip(add_names, add_types)],
        mask=pa.array(~add_valid))
    rm_type = pa.struct([("path", pa.string()), ("deletionTimestamp", pa.int64()),
                         ("dataChange", pa.bool_()), ("extendedFileMetadata", pa.bool_()),
                         ("partitionValues", mt), ("size", pa.int64()), ("tags", mt)])
    txn_type = pa.struct([("appId", pa.string()), ("version", pa.int64()), ("lastUpdated", pa.int64())])
    md = metadata_dict(ncols)
    fmt_type = pa.struct([("provider", pa.string()), ("options", mt)])
    md_type = pa.struct([("id", pa.string()), ("name", pa.string()), ("description", pa.string()),
                         ("format", fmt_type), ("schemaString", pa.string()),
                         ("partitionColumns", pa.list_(pa.string())), ("configuration", mt),
                         ("createdTime", pa.int64())])
    md_rows = [None, {"id": md["id"], "name": None, "description": None,
                      "format": {"provider": "parquet", "options": []},
                      "schemaString": md["schemaString"], "partitionColumns": md["partitionColumns"],
                      "configuration": [], "createdTime": md["createdTime"]}]
    prot_type = pa.struct([("minReaderVersion", pa.int32()), ("minWriterVersion", pa.int32())])
    if head:
        md_struct = pa.concat_arrays([pa.array(md_rows, md_type), pa.nulls(n, md_type)])
        prot_struct = pa.concat_arrays([pa.array([{"minReaderVersion": 1, "minWriterVersion": 2}], prot_type),
                                        pa.nulls(n + 1, prot_type)])
    else:
        md_struct, prot_struct = pa.nulls(n, md_type), pa.nulls(n, prot_type)
    table = pa.Table.from_arrays([pa.nulls(nrows, txn_type), add_struct, pa.nulls(nrows, rm_type),
                                  md_struct, prot_struct],
                                 names=["txn", "add", "remove", "metaData", "protocol"])
    pq.write_table(table, path, compression=compression, use_dictionary=use_dictionary, version="1.0",
                   data_page_version=data_page_version, row_group_size=row_group_size,
                   data_page_size=data_page_size, write_statistics=False)
    return nrows


def write_checkpoint_records(path: str, protocol: dict, metadata: dict, adds: list, removes: list = (),
                             txns: list = (), row_group_size: int = 1 << 20, use_dictionary: bool = True,
                             data_page_version: str = "1.0", data_page_size: int = 1 << 20) -> int:
    """Checkpoint with the reference's column layout from explicit action records (edge-case
    corpora: any partitionValues / tags maps, nulls). Rows: protocol, metaData, txns, adds, removes
    (protocol / metadata None: no such row, as in DeltaLogSuite's checkpoints missing an action)."""
    pa, _ = _pa()
    import pyarrow.parquet as pq
    mt = pa.map_(pa.string(), pa.string())
    add_type = pa.struct([("path", pa.string()), ("partitionValues", mt), ("size", pa.int64()),
                          ("modificationTime", pa.int64()), ("dataChange", pa.bool_()), ("tags", mt),
                          ("stats", pa.string())])
    rm_type = pa.struct([("path", pa.string()), ("deletionTimestamp", pa.int64()),
                         ("dataChange", pa.bool_()), ("extendedFileMetadata", pa.bool_()),
                         ("partitionValues", mt), ("size", pa.int64()), ("tags", mt)])
    txn_type = pa.struct([("appId", pa.string()), ("version", pa.int64()), ("lastUpdated", pa.int64())])
    fmt_type = pa.struct([("provider", pa.string()), ("options", mt)])
    md_type = pa.struct([("id", pa.string()), ("name", pa.string()), ("description", pa.string()),
                         ("format", fmt_type), ("schemaString", pa.string()),
                         ("partitionColumns", pa.list_(pa.string())), ("configuration", mt),
                         ("createdTime", pa.int64())])
    prot_type = pa.struct([("minReaderVersion", pa.int32()), ("minWriterVersion", pa.int32())])

    def m(d):
        return None if d is None else list(d.items())

    rows = []
    if protocol is not None:
        rows.append({"protocol": protocol})
    if metadata is not None:
        md = dict(metadata)
        rows.append({"metaData": {"id": md["id"], "name": md.get("name"), "description": md.get("description"),
                                  "format": {"provider": md.get("format", {}).get("provider", "parquet"),
                                             "options": m(md.get("format", {}).get("options") or {})},
                                  "schemaString": md["schemaString"],
                                  "partitionColumns": md.get("partitionColumns", []),
                                  "configuration": m(md.get("configuration") or {}),
                                  "createdTime": md.get("createdTime")}})
    rows += [{"txn": t} for t in txns]
    for a in adds:
        rows.append({"add": dict(path=a["path"], partitionValues=m(a.get("partitionValues")), size=a.get("size", 0),
                                 modificationTime=a.get("modificationTime", 0), dataChange=False,
                                 tags=m(a.get("tags")), stats=a.get("stats"))})
    for r in removes:
        rows.append({"remove": dict(path=r["path"], deletionTimestamp=r.get("deletionTimestamp"), dataChange=False,
                                    extendedFileMetadata=r.get("extendedFileMetadata", False),
                                    partitionValues=m(r.get("partitionValues")), size=r.get("size"),
                                    tags=m(r.get("tags")))})
    cols = {}
    for name, typ in (("txn", txn_type), ("add", add_type), ("remove", rm_type), ("metaData", md_type),
                      ("protocol", prot_type)):
        cols[name] = pa.array([r.get(name) for r in rows], typ)
    table = pa.Table.from_arrays(list(cols.values()), names=list(cols))
    pq.write_table(table, path, compression="snappy", use_dictionary=use_dictionary, version="1.0",
                   data_page_version=data_page_version, row_group_size=row_group_size,
                   data_page_size=data_page_size, write_statistics=False)
    return len(rows)


# ----------------------------------------------------------------------------------------------
# Config builders
# ----------------------------------------------------------------------------------------------
@dataclass
class ChurnSpec:
    ckpt_files: int            # live files in the checkpoint (0 = no checkpoint)
    ckpt_version: int
    n_deltas: int
    removes_per_delta: int
    adds_per_delta: int
    readd_frac: float          # fraction of adds that re-add earlier-removed paths
    ncols: int = 2
    n_at_cutoff: int = 0       # removes placed exactly at the cutoff (must be dropped)
    init_adds: int = 0         # no-checkpoint mode: adds in v0 (with protocol+metadata)
    ckpt_parts: int = 1        # > 1: a multi-part checkpoint (FileNames.checkpointFileWithParts)


_FORK_STATE = None


def _write_parts_worker(job):
    """One worker of build_table's parallel multi-part checkpoint write (forked: the pool is shared)."""
    pool, ids, per, kw = _FORK_STATE
    out = []
    for k, cp in job:
        out.append((k, write_checkpoint(cp, pool, ids[k * per:(k + 1) * per], head=k == 0, **kw),
                    os.path.getsize(cp)))
    return out


def _pick_live(rng, state, next_id, k):
    """k distinct live ids. Small picks from a large pool (config 5's streaming tail: 2 removes per
    commit over 50M files) sample and reject instead of listing the live set on every commit."""
    if 0 < k and k * 1000 < next_id:
        for _ in range(8):
            cand = np.unique(rng.integers(0, next_id, 4 * k + 16))
            cand = cand[state[cand] == 1]
            if len(cand) >= k:
                return rng.permutation(cand)[:k]
    live = np.flatnonzero(state == 1)
    return rng.choice(live, size=min(k, len(live)), replace=False)


def build_table(table_dir: str, spec: ChurnSpec, seed: int, checkpoint_with_parsed=False,
                data_page_size: int = 1 << 20, keep_ids: bool = True, compression: str = "snappy",
                data_page_version: str = "1.0", row_group_size: int = 1 << 20,
                use_dictionary: bool = True, workers: int = 1) -> Expected:
    rng = np.random.default_rng(seed)
    log = os.path.join(table_dir, "_delta_log")
    os.makedirs(log, exist_ok=True)
    total_new = spec.ckpt_files + spec.init_adds + spec.n_deltas * spec.adds_per_delta
    pool = FilePool(rng, max(total_new, 1), spec.ncols)
    state = np.zeros(len(pool), np.int8)   # 0 never seen, 1 live, 2 removed
    delts = np.zeros(len(pool), np.int64)
    n_actions = n_file_actions = json_bytes = ckpt_bytes = 0
    window0 = T0 + 30 * DAY_MS           # deletionTimestamp window [window0, window0 + 14 days)
    cutoff = window0 + 7 * DAY_MS
    version = 0
    if spec.ckpt_files:
        version = spec.ckpt_version
        ids = np.arange(spec.ckpt_files)
        next_id = spec.ckpt_files
        state[ids] = 1
        parts = max(1, spec.ckpt_parts)
        nrows = 0
        per = (spec.ckpt_files + parts - 1) // parts
        kw = dict(ncols=spec.ncols, version=version, with_parsed=checkpoint_with_parsed,
                  data_page_size=data_page_size, compression=compression, data_page_version=data_page_version,
                  row_group_size=row_group_size, use_dictionary=use_dictionary)
        names = [os.path.join(log, "%020d.checkpoint.parquet" % version if parts == 1 else
                              "%020d.checkpoint.%010d.%010d.parquet" % (version, k + 1, parts))
                 for k in range(parts)]
        jobs = [[(k, names[k]) for k in range(w, parts, max(1, workers))] for w in range(max(1, workers))]
        global _FORK_STATE
        _FORK_STATE = (pool, ids, per, kw)
        if workers > 1 and parts > 1:
            import multiprocessing as mp
            with mp.get_context("fork").Pool(min(workers, parts)) as P:
                results = [r for rs in P.map(_write_parts_worker, [j for j in jobs if j]) for r in rs]
        else:
            results = _write_parts_worker([(k, names[k]) for k in range(parts)])
        _FORK_STATE = None
        for _, rows, size in results:
            nrows += rows
            ckpt_bytes += size
        n_actions += nrows
        n_file_actions += spec.ckpt_files
        with open(os.path.join(log, "_last_checkpoint"), "w") as f:
            f.write('{"version":%d,"size":%d%s}\n' % (version, nrows, ',"parts":%d' % parts if parts > 1 else ""))
        # an earlier commit at the checkpoint version (listed, not replayed)
        with open(os.path.join(log, delta_name(version)), "w") as f:
            f.write(commit_info_line(version) + "\n")
    else:
        ids = np.arange(spec.init_adds)
        next_id = spec.init_adds
        state[ids] = 1
        head = "\n".join([commit_info_line(0), protocol_line(), metadata_line(spec.ncols)]) + "\n"
        body = head.encode() + _text_bytes(add_lines(pool, ids, T0 + np.arange(len(ids))))
        with open(os.path.join(log, delta_name(0)), "wb") as f:
            f.write(body)
        json_bytes += len(body)
        n_actions += 3 + len(ids)
        n_file_actions += len(ids)
    removed_pool = np.zeros(0, np.int64)
    at_cutoff_left = spec.n_at_cutoff
    for _ in range(spec.n_deltas):
        version += 1
        rm_ids = _pick_live(rng, state, next_id, spec.removes_per_delta)
        ts = rng.integers(window0, window0 + 14 * DAY_MS, len(rm_ids), dtype=np.int64)
        if at_cutoff_left:
            k = min(at_cutoff_left, len(ts))
            ts[:k] = cutoff
            at_cutoff_left -= k
        n_readd = int(spec.adds_per_delta * spec.readd_frac) if len(removed_pool) else 0
        n_readd = min(n_readd, len(removed_pool))
        if n_readd:
            pick = rng.choice(len(removed_pool), size=n_readd, replace=False)
            readd = removed_pool[pick]
            keep = np.ones(len(removed_pool), bool)
            keep[pick] = False
            removed_pool = removed_pool[keep]
        else:
            readd = np.zeros(0, np.int64)
        n_new = spec.adds_per_delta - n_readd
        new = np.arange(next_id, next_id + n_new)
        next_id += n_new
        add_ids = np.concatenate([readd, new]).astype(np.int64)
        mt0 = T0 + version * 60000
        body = (commit_info_line(version, "OPTIMIZE" if spec.removes_per_delta else "WRITE") + "\n").encode()
        body += _text_bytes(remove_lines(pool, rm_ids, ts))
        body += _text_bytes(add_lines(pool, add_ids, mt0 + np.arange(len(add_ids))))
        with open(os.path.join(log, delta_name(version)), "wb") as f:
            f.write(body)
        json_bytes += len(body)
        state[rm_ids] = 2
        delts[rm_ids] = ts
        state[add_ids] = 1
        removed_pool = np.concatenate([removed_pool, rm_ids.astype(np.int64)])
        n_actions += 1 + len(rm_ids) + len(add_ids)
        n_file_actions += len(rm_ids) + len(add_ids)
    live_ids = np.flatnonzero(state == 1)
    tomb_ids = np.flatnonzero((state == 2) & (delts > cutoff))
    return Expected(version=version, min_file_retention_timestamp=cutoff,
                    num_files=len(live_ids), size_in_bytes=int(pool.size[live_ids].sum()),
                    num_removes=len(tomb_ids), num_actions=n_actions, num_file_actions=n_file_actions,
                    live_ids=live_ids if keep_ids else None, tomb_ids=tomb_ids if keep_ids else None,
                    json_bytes=json_bytes, checkpoint_bytes=ckpt_bytes)


def config_spec(config: int, scale: float = 1.0) -> ChurnSpec:
    """BASELINE.json configs; `scale` shrinks file counts for tests."""
    s = lambda x: max(1, int(round(x * scale)))
    if config == 1:
        return ChurnSpec(ckpt_files=0, ckpt_version=0, n_deltas=99, removes_per_delta=0,
                         adds_per_delta=s(100), readd_frac=0.0, ncols=2, init_adds=s(100))
    if config == 2:
        return ChurnSpec(ckpt_files=s(1_000_000), ckpt_version=100, n_deltas=10,
                         removes_per_delta=s(5000), adds_per_delta=s(5000), readd_frac=0.0, ncols=2)
    if config == 3:
        return ChurnSpec(ckpt_files=s(10_000_000), ckpt_version=1000, n_deltas=30,
                         removes_per_delta=s(100_000), adds_per_delta=s(100_000), readd_frac=0.5,
                         ncols=2, n_at_cutoff=min(1000, s(1000)))
    if config == 4:  # 100 parts of 1M rows at full scale (at least 2 parts when scaled down)
        files = s(100_000_000)
        return ChurnSpec(ckpt_files=files, ckpt_version=1000, n_deltas=0, removes_per_delta=0, adds_per_delta=0,
                         readd_frac=0.0, ncols=4, ckpt_parts=min(100, max(2, files // 1000)))
    if config == 5:  # streaming tail: 10k commits of 3 adds + 2 removes over a 50M-file checkpoint
        files = s(50_000_000)
        return ChurnSpec(ckpt_files=files, ckpt_version=100, n_deltas=min(10_000, max(20, s(10_000))),
                         removes_per_delta=2, adds_per_delta=3, readd_frac=0.0, ncols=2,
                         ckpt_parts=min(50, max(1, files // 1_000_000)))
    raise ValueError(config)


def build_config(config: int, table_dir: str, scale: float = 1.0, seed: Optional[int] = None,
                 **kw) -> Expected:
    seed = BASE_SEED + config if seed is None else seed
    return build_table(table_dir, config_spec(config, scale), seed, **kw)


def config4_selected(table_dir: str, scale: float = 1.0, seed: Optional[int] = None) -> int:
    """Files config 4's predicate keeps: p0 >= DATE'2020-03-01' AND p0 < DATE'2020-06-01'
    AND p1 IN (1..100) AND p2 = 'w17' AND p3 = true, counted from the generator's pool by construction."""
    seed = BASE_SEED + 4 if seed is None else seed
    spec = config_spec(4, scale)
    pool = FilePool(np.random.default_rng(seed), spec.ckpt_files, spec.ncols)
    keep = ((pool.p0 >= 60) & (pool.p0 < 152) & (pool.p1 >= 1) & (pool.p1 <= 100) & (pool.p2 == 17)
            & ~pool.p2null & (pool.p3 == 1))
    return int(keep.sum())


def config4_predicate():
    """Config 4's filter as conjuncts in the predicate-tree form of delta_amd/predicates.py."""
    col = lambda c: ("col", c)
    lit = lambda t, v: ("lit", t, v)
    return [(">=", col("p0"), lit("date", "2020-03-01")), ("<", col("p0"), lit("date", "2020-06-01")),
            ("in", col("p1"), [lit("integer", v) for v in range(1, 101)]), ("=", col("p2"), lit("string", WORDS[17])),
            ("=", col("p3"), lit("boolean", True))]


if __name__ == "__main__":  # python -m delta_amd.testing.synth <config> <table_dir> [scale] [workers]
    import sys
    cfg, out = int(sys.argv[1]), sys.argv[2]
    sc = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    nw = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    e = build_config(cfg, out, scale=sc, keep_ids=False, workers=nw)
    d = {k: getattr(e, k) for k in ("version", "min_file_retention_timestamp", "num_files", "size_in_bytes",
                                    "num_removes", "num_actions", "num_file_actions", "json_bytes", "checkpoint_bytes")}
    d["n_deltas"] = config_spec(cfg, sc).n_deltas
    if cfg == 4:
        d["selected"] = config4_selected(out, sc)
    with open(os.path.join(out, "expected.json"), "w") as f:
        json.dump(d, f)
    print(json.dumps(d))
