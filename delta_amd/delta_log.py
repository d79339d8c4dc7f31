"""Host-side mirror of the reference's DeltaLog / Snapshot API over the MI355X replay engine.

Same names, argument meaning and error behaviour as the reference for this path:
  DeltaLog.for_table            <- DeltaLog.forTable (D/DeltaLog.scala:390-475)
  DeltaLog.update / snapshot    <- SnapshotManagement.update (D/SnapshotManagement.scala:244-339)
  DeltaLog.get_snapshot_at      <- SnapshotManagement.getSnapshotAt (:342-360)
  DeltaLog.min_file_retention_timestamp <- D/DeltaLog.scala:109-120
  Snapshot.all_files/tombstones <- D/Snapshot.scala:193-204 (dataChange forced false)
  Snapshot.num_of_files etc.    <- computedState (D/Snapshot.scala:136-186)
  Snapshot.files_for_scan       <- PartitionFiltering.filesForScan (D/PartitionFiltering.scala:27-42)
  InMemoryLogReplay             <- D/actions/InMemoryLogReplay.scala:35-77 (append/checkpoint)

All replay work runs in libdeltareplay on the GPU; this module only does control flow.
D/ = core/src/main/scala/org/apache/spark/sql/delta/ of the reference checkout.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import json
import os
import re
import threading
import time
import weakref
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from . import _native as N



def _owned_bytes(lib, buf, n: int) -> memoryview:
    """A read-only bytes view of a library-allocated block (a checkpoint part: pinned host memory)
    without copying it; the block goes back to the library (dr_free) when the last view of it is
    dropped."""
    if not n:
        lib.dr_free(C.cast(buf, C.c_void_p))
        return memoryview(b"")
    arr = (C.c_uint8 * n).from_address(C.cast(buf, C.c_void_p).value)
    weakref.finalize(arr, lib.dr_free, C.c_void_p(C.cast(buf, C.c_void_p).value))
    return memoryview(arr).cast("B").toreadonly()

class DeltaError(Exception):
    """Carries the reference's exception class name (`kind`) and the C status."""

    KIND = {3: "FileNotFoundException", 4: "FileNotFoundException", 5: "IllegalStateException",
            6: "IllegalStateException", 7: "IllegalArgumentException", 8: "IllegalStateException",
            9: "IllegalStateException", 10: "IllegalStateException", 11: "IllegalStateException",
            16: "IllegalStateException", 19: "AssertionError"}

    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status
        self.code = N.STATUS.get(status, str(status))
        self.kind = self.KIND.get(status, "RuntimeException")


# ---- clocks (org.apache.spark.util.Clock / ManualClock as used by DeltaRetentionSuite) ---------
class SystemClock:
    def get_time_millis(self) -> int:
        return int(time.time() * 1000)


class ManualClock:
    def __init__(self, t: int = 0):
        self.t = int(t)

    def get_time_millis(self) -> int:
        return self.t

    def advance(self, ms: int) -> None:
        self.t += int(ms)


# ---- engine (one dr_ctx per thread and device) --------------------------------------------------
class Engine:
    _tls = threading.local()

    def __init__(self, device: int = 0):
        self.lib = N.lib()
        self.ctx = C.c_void_p()
        rc = self.lib.dr_ctx_create(device, C.byref(self.ctx))
        if rc != N.DR_OK:
            raise DeltaError(rc, "cannot open HIP device %d (libdeltareplay needs an MI355X GPU)" % device)
        self.device = device
        # the library serialises the calls on one dr_ctx itself (ABI 4, include/deltareplay.h); this
        # lock also keeps a multi-call sequence (set an option, then replay) of one thread together
        self.lock = threading.RLock()

    @classmethod
    def get(cls, device: int = 0) -> "Engine":
        d = getattr(cls._tls, "engines", None)
        if d is None:
            d = cls._tls.engines = {}
        if device not in d:
            d[device] = Engine(device)
        return d[device]

    def check(self, rc: int) -> None:
        if rc != N.DR_OK:
            raise DeltaError(rc, self.lib.dr_last_error(self.ctx).decode("utf-8", "replace"))

    def set_option(self, name: str, value: int) -> int:
        """dr_ctx_set_option (include/deltareplay.h enum dr_option, by its lower-case name without
        DR_OPT_): the context's per-session configuration, as the reference reads DeltaSQLConf from
        the session (D/sources/DeltaSQLConf.scala:29). Returns the previous value."""
        with self.lock:
            old = self.get_option(name)
            self.check(self.lib.dr_ctx_set_option(self.ctx, N.OPTIONS[name], int(value)))
        return old

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        self.check(self.lib.dr_ctx_get_option(self.ctx, N.OPTIONS[name], C.byref(v)))
        return v.value

    @contextlib.contextmanager
    def options(self, **opts):
        """Sets context options for the body of a `with` and restores them after (tests)."""
        old = {}
        try:
            for k, v in opts.items():
                old[k] = self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    def set_timing(self, on: bool, only: Optional[str] = None) -> None:
        """dr_set_timing (+ dr_set_timing_only: events around one kernel only)."""
        self.check(self.lib.dr_set_timing_only(self.ctx, (only or "").encode()))
        self.check(self.lib.dr_set_timing(self.ctx, 1 if on else 0))

    def last_timings(self) -> Dict[str, float]:
        cap = 1024
        names = C.create_string_buffer(64 * cap)
        ms = (C.c_float * cap)()
        n = C.c_int32()
        self.check(self.lib.dr_last_timings(self.ctx, names, 64 * cap, ms, cap, C.byref(n)))
        parts = names.raw.split(b"\0", min(n.value, cap))  # only the names written (the bench calls this per timed step)
        out: Dict[str, float] = {}
        for i in range(min(n.value, cap)):
            k = parts[i].decode()
            out[k] = out.get(k, 0.0) + float(ms[i])
        return out

    # staging / replay -------------------------------------------------------------------------
    def stage_log(self, log_path: str, version: int = -1) -> "Staged":
        h = C.c_void_p()
        with self.lock:
            self.check(self.lib.dr_stage_log(self.ctx, log_path.encode(), int(version), C.byref(h)))
        return Staged(self, h)

    def stage_files(self, files: Sequence[Tuple[int, int, int, bytes]], log_path: Optional[str] = None,
                    names: Optional[Sequence[str]] = None) -> "Staged":
        """dr_stage; with `log_path` and the files' `names`, dr_stage_named (every named file must
        sit in log_path: assertLogBelongsToTable, D/Snapshot.scala:334-345)."""
        arr = (N.dr_file * max(len(files), 1))()
        keep = []
        for i, (version, kind, part, data) in enumerate(files):
            buf = C.create_string_buffer(data, len(data))
            keep.append(buf)
            arr[i] = N.dr_file(version, kind, part, C.cast(buf, C.c_void_p), len(data))
        h = C.c_void_p()
        with self.lock:
            if log_path is None:
                self.check(self.lib.dr_stage(self.ctx, arr, len(files), C.byref(h)))
            else:
                nm = (C.c_char_p * max(len(files), 1))(*[(n or "").encode() for n in (names or [""] * len(files))])
                self.check(self.lib.dr_stage_named(self.ctx, log_path.encode(), arr, nm, len(files), C.byref(h)))
        return Staged(self, h)

    @staticmethod
    def comm_unique_id() -> bytes:
        """dr_comm_unique_id: the 128-byte RCCL id one rank creates and shares with the others."""
        buf = C.create_string_buffer(128)
        rc = N.lib().dr_comm_unique_id(buf)
        if rc != N.DR_OK:
            raise DeltaError(rc, "dr_comm_unique_id failed (%s)" % N.STATUS.get(rc, rc))
        return buf.raw

    @staticmethod
    def comm_loopback_id() -> bytes:
        """dr_comm_loopback_id (test hook): an id whose communicator is an in-process loopback -- the
        ranks are threads of this process, the collectives device copies at a barrier."""
        buf = C.create_string_buffer(128)
        rc = N.lib().dr_comm_loopback_id(buf)
        if rc != N.DR_OK:
            raise DeltaError(rc, "dr_comm_loopback_id failed (%s)" % N.STATUS.get(rc, rc))
        return buf.raw

    def comm(self, uid: bytes, world: int, rank: int) -> "Comm":
        """dr_comm_create: this rank's RCCL communicator (collective over the `world` ranks)."""
        h = C.c_void_p()
        with self.lock:
            self.check(self.lib.dr_comm_create(self.ctx, uid, int(world), int(rank), C.byref(h)))
        return Comm(self, h)

    def log_segment(self, log_path: str, version: int = -1):
        need = C.c_uint64()
        ver = C.c_int64()
        self.check(self.lib.dr_log_segment(self.ctx, log_path.encode(), int(version), None, 0,
                                           C.byref(need), C.byref(ver)))
        buf = C.create_string_buffer(need.value + 1)
        self.check(self.lib.dr_log_segment(self.ctx, log_path.encode(), int(version), buf, need.value + 1,
                                           C.byref(need), C.byref(ver)))
        files = []
        for line in buf.value.decode().splitlines():
            kind, v, part, name = line.split(" ", 3)
            files.append((int(kind), int(v), int(part), name))
        return ver.value, files


class Comm:
    """An RCCL communicator of the library's in-process sharded replay (dr_replay_sharded)."""

    def __init__(self, eng: "Engine", h):
        self.eng = eng
        self.h = h

    def replay_sharded(self, staged: "Staged", min_file_retention_timestamp: int, validate: bool = True) -> "State":
        st = C.c_void_p()
        flags = 0 if validate else N.DR_FLAG_NO_VALIDATION
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_replay_sharded(self.h, staged.h, int(min_file_retention_timestamp), flags,
                                                          C.byref(st)))
        return State(self.eng, st)

    def release(self) -> None:
        if self.h:
            self.eng.lib.dr_comm_release(self.h)
            self.h = None


class Staged:
    def __init__(self, eng: Engine, handle: C.c_void_p):
        self.eng, self.h = eng, handle

    def bytes(self) -> Tuple[int, int]:
        j, c = C.c_uint64(), C.c_uint64()
        self.eng.check(self.eng.lib.dr_staged_bytes(self.h, C.byref(j), C.byref(c)))
        return j.value, c.value

    def plan(self) -> Dict[str, int]:
        out = (C.c_uint64 * 16)()
        n = C.c_int32()
        self.eng.check(self.eng.lib.dr_staged_plan(self.h, out, 16, C.byref(n)))
        names = ["json_bytes", "checkpoint_bytes", "checkpoint_rows", "pages", "pages_compressed_bytes",
                 "pages_decompressed_bytes", "dict_entries", "snappy_in_bytes", "snappy_out_bytes",
                 "snappy_chunks", "snappy_blocks", "snappy_elements", "copy_bytes", "json_lines"]
        return {names[i]: int(out[i]) for i in range(n.value)}

    def replay(self, min_file_retention_timestamp: int, validate: bool = True, reducer: str = "lds") -> "State":
        """`reducer` is a test hook: "reduce64" / "exact" force every hash bucket through the 64-bit-key
        or the O(m^2) fallback reducer instead of the LDS rkey table."""
        st = C.c_void_p()
        flags = (0 if validate else N.DR_FLAG_NO_VALIDATION) | {
            "lds": 0, "reduce64": N.DR_FLAG_REDUCE64, "exact": N.DR_FLAG_EXACT_REDUCE}[reducer]
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_replay_staged(self.eng.ctx, self.h, int(min_file_retention_timestamp),
                                                         flags, C.byref(st)))
        return State(self.eng, st)

    def parse_lines(self) -> List[dict]:
        """dr_parse_commits: K1's reading of every staged commit line -- {"version", "kind",
        "path" (raw JSON string body, bytes) or None, "escaped", "size", "deletionTimestamp"}."""
        lines = N.dr_lines()
        h = C.c_void_p()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_parse_commits(self.eng.ctx, self.h, C.byref(h), C.byref(lines)))
        try:
            n = lines.n
            raw = C.string_at(lines.bytes, lines.nbytes) if lines.nbytes else b""
            out = []
            for i in range(n):
                k, f = lines.kind[i], lines.flags[i]
                rec = {"version": lines.version[i], "kind": k,
                       "line": raw[lines.line_off[i]:lines.line_off[i] + lines.line_len[i]]}
                if k in (1, 2):
                    po = lines.path_off[i]
                    rec["path"] = None if f & 8 else raw[po:po + lines.path_len[i]]
                    rec["escaped"] = bool(f & 4)
                    rec["size"] = lines.size[i]
                    rec["deletionTimestamp"] = lines.deletion_timestamp[i] if f & 1 else None
                out.append(rec)
            return out
        finally:
            self.eng.lib.dr_parsed_release(h)

    def release(self) -> None:
        if self.h:
            with self.eng.lock:
                self.eng.lib.dr_staged_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


def _arr(ptr, n):
    return [ptr[i] for i in range(n)]


class State:
    """The reconstructed state resident in HBM (the reference's cached `state` Dataset)."""

    def __init__(self, eng: Engine, handle: C.c_void_p):
        self.eng, self.h = eng, handle
        c = N.dr_counts()
        eng.check(eng.lib.dr_state_counts(handle, C.byref(c)))
        self.counts = {f: getattr(c, f) for f, _ in N.dr_counts._fields_}
        p = C.c_char_p()
        n = C.c_uint64()
        eng.check(eng.lib.dr_state_nonfile_json(handle, C.byref(p), C.byref(n)))
        self._nonfile_text = C.string_at(p, n.value) if n.value else b""
        self._nonfile = None

    def materialize(self) -> int:
        """dr_state_materialize: every field of both sides extracted on the device and kept resident
        (the reference's cached SingleAction rows); returns the device bytes they hold."""
        b = C.c_uint64()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_materialize(self.h, C.byref(b)))
        return b.value

    def local_counts(self) -> Dict[str, int]:
        """dr_state_local_counts: a library-sharded rank's own counters before the all-reduce (its
        parsed and reduced actions); the table-wide `counts` for any other state."""
        c = N.dr_counts()
        self.eng.check(self.eng.lib.dr_state_local_counts(self.h, C.byref(c)))
        return {f: getattr(c, f) for f, _ in N.dr_counts._fields_}

    @property
    def nonfile(self) -> List[dict]:
        """protocol / metaData / txn winners (dr_state_nonfile_json), decoded on first use."""
        if self._nonfile is None:
            text = self._nonfile_text.decode("utf-8")
            self._nonfile = [json.loads(l) for l in text.splitlines() if l.strip()]
        return self._nonfile

    @nonfile.setter
    def nonfile(self, v: List[dict]) -> None:
        self._nonfile = v

    def set_nonfile_json(self, lines: str, validate: bool = True) -> None:
        """dr_state_set_nonfile_json: a sharded state's table-wide protocol / metaData / txn winners
        from every rank's local winners (one action per line, rank order)."""
        raw = lines.encode("utf-8")
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_set_nonfile_json(self.h, raw, len(raw),
                                                                  0 if validate else N.DR_FLAG_NO_VALIDATION))
        p = C.c_char_p()
        n = C.c_uint64()
        self.eng.check(self.eng.lib.dr_state_nonfile_json(self.h, C.byref(p), C.byref(n)))
        text = C.string_at(p, n.value).decode("utf-8") if n.value else ""
        self.nonfile = [json.loads(l) for l in text.splitlines() if l.strip()]

    def apply(self, tail: "Staged", min_file_retention_timestamp: int, validate: bool = True) -> "State":
        """dr_state_apply: this state extended by the staged commit files of the following
        versions (no re-parse of this state's segment); a new State."""
        st = C.c_void_p()
        flags = 0 if validate else N.DR_FLAG_NO_VALIDATION
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_apply(self.eng.ctx, self.h, tail.h,
                                                       int(min_file_retention_timestamp), flags, C.byref(st)))
        return State(self.eng, st)

    def check_checksum(self, crc_line: bytes) -> Optional[str]:
        """checkMismatch (D/Checksum.scala:178-191): None when the counters match, else the
        mismatch text. Raises ValueError when the line is not a VersionChecksum (no validation)."""
        buf = C.create_string_buffer(1024)
        n = C.c_uint64()
        with self.eng.lock:
            rc = self.eng.lib.dr_state_check_checksum(self.h, crc_line, len(crc_line), buf, 1024, C.byref(n))
        if rc == N.DR_E_NO_CHECKSUM:
            raise ValueError("unparseable checksum")
        if rc == N.DR_E_CHECKSUM:
            if n.value >= 1024:
                buf = C.create_string_buffer(n.value + 1)
                self.eng.lib.dr_state_check_checksum(self.h, crc_line, len(crc_line), buf, n.value + 1, C.byref(n))
            return buf.value.decode("utf-8")
        self.eng.check(rc)
        return None

    def record_sums(self) -> Tuple[int, int]:
        """dr_state_record_sums: (live, tombstone) order-free full-record checksums, computed on the
        device (same definition as oracle.delta_oracle.record_hash)."""
        a, b = C.c_uint64(), C.c_uint64()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_record_sums(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def record_hashes(self, which: int):
        """dr_state_record_hashes: every record's hash of one side (numpy uint64, export order)."""
        import numpy as np
        lc = self.local_counts()  # a sharded rank's own rows (the table-wide counts otherwise)
        n = lc["num_files"] if which == N.DR_LIVE else lc["num_removes"]
        out = np.zeros(max(int(n), 1), dtype=np.uint64)
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_record_hashes(self.h, which, out.ctypes.data, int(n)))
        return out[:int(n)]

    def export(self, which: int) -> List[dict]:
        with self.eng.lock:
            return self._export(which)

    def _export(self, which: int) -> List[dict]:
        e = N.dr_export()
        self.eng.check(self.eng.lib.dr_state_export(self.h, which, C.byref(e)))
        n = e.n
        out = []
        if n == 0:
            return out

        def strs(off, data, count):
            o = _arr(off, count + 1)
            raw = C.string_at(data, o[-1]) if o[-1] else b""
            return [raw[o[i]:o[i + 1]].decode("utf-8") for i in range(count)]

        paths = strs(e.path_off, e.path_bytes, n)
        sizes = _arr(e.size, n)
        stats = strs(e.stats_off, e.stats_bytes, n)
        stats_null = _arr(e.stats_null, n)

        def maps(entry_off, map_null, koff, kbytes, voff, vbytes, vnull):
            eo = _arr(entry_off, n + 1)
            m = eo[-1]
            ks = strs(koff, kbytes, m) if m else []
            vs = strs(voff, vbytes, m) if m else []
            vn = _arr(vnull, m) if m else []
            nulls = _arr(map_null, n)
            res = []
            for i in range(n):
                if nulls[i]:
                    res.append(None)
                    continue
                res.append({ks[j]: (None if vn[j] else vs[j]) for j in range(eo[i], eo[i + 1])})
            return res

        pvs = maps(e.pv_entry_off, e.pv_null, e.pv_key_off, e.pv_key_bytes, e.pv_val_off, e.pv_val_bytes,
                   e.pv_val_null)
        tags = maps(e.tags_entry_off, e.tags_null, e.tags_key_off, e.tags_key_bytes, e.tags_val_off,
                    e.tags_val_bytes, e.tags_val_null)
        if which == N.DR_LIVE:
            mt = _arr(e.modification_time, n)
            for i in range(n):
                out.append({"path": paths[i], "partitionValues": pvs[i], "size": sizes[i],
                            "modificationTime": mt[i], "dataChange": False,
                            "stats": None if stats_null[i] else stats[i], "tags": tags[i]})
        else:
            dt = _arr(e.deletion_timestamp, n)
            dv = _arr(e.deletion_timestamp_valid, n)
            efm = _arr(e.extended_file_metadata, n)
            for i in range(n):
                out.append({"path": paths[i], "deletionTimestamp": dt[i] if dv[i] else None,
                            "dataChange": False, "extendedFileMetadata": bool(efm[i]),
                            "partitionValues": pvs[i], "size": sizes[i], "tags": tags[i]})
        return out

    # dr_export's columns: (field, element type, count kind) -- count kinds: n rows, n+1 offsets, e
    # entries, e+1 entry offsets, or the byte total of the named offset column
    _COLS = [("path_off", "i8", "n1"), ("path_bytes", "u1", "path_off"), ("size", "i8", "n"),
             ("modification_time", "i8", "n"), ("deletion_timestamp", "i8", "n"),
             ("deletion_timestamp_valid", "u1", "n"), ("extended_file_metadata", "u1", "n"),
             ("stats_off", "i8", "n1"), ("stats_bytes", "u1", "stats_off"), ("stats_null", "u1", "n"),
             ("pv_entry_off", "i8", "n1"), ("pv_null", "u1", "n"), ("pv_key_off", "i8", "pv1"),
             ("pv_key_bytes", "u1", "pv_key_off"), ("pv_val_off", "i8", "pv1"), ("pv_val_bytes", "u1", "pv_val_off"),
             ("pv_val_null", "u1", "pv"), ("tags_entry_off", "i8", "n1"), ("tags_null", "u1", "n"),
             ("tags_key_off", "i8", "tg1"), ("tags_key_bytes", "u1", "tags_key_off"),
             ("tags_val_off", "i8", "tg1"), ("tags_val_bytes", "u1", "tags_val_off"), ("tags_val_null", "u1", "tg")]

    @staticmethod
    def _columns(e) -> Dict[str, "object"]:
        """numpy views of a dr_export's columns (valid while their owner lives)."""
        import numpy as np
        n = e.n
        out = {}

        def view(name, dt, cnt):
            ptr = getattr(e, name)
            if cnt == 0 or not ptr:
                return np.zeros(0, dtype=dt)
            ct = C.c_int64 if dt == "i8" else C.c_uint8
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(cnt,))
        out["path_off"] = view("path_off", "i8", n + 1)
        out["pv_entry_off"] = view("pv_entry_off", "i8", n + 1)
        out["tags_entry_off"] = view("tags_entry_off", "i8", n + 1)
        out["stats_off"] = view("stats_off", "i8", n + 1)
        npv = int(out["pv_entry_off"][-1]) if n else 0
        ntg = int(out["tags_entry_off"][-1]) if n else 0
        cnts = {"n": n, "n1": n + 1, "pv": npv, "pv1": npv + 1, "tg": ntg, "tg1": ntg + 1}
        for name, dt, kind in State._COLS:
            if name in out:
                continue
            if kind in cnts:
                out[name] = view(name, dt, cnts[kind])
        for name, dt, kind in State._COLS:
            if name not in out:
                offs = out[kind]
                out[name] = view(name, dt, int(offs[-1]) if len(offs) else 0)
        return out

    def export_columns(self, which: int) -> Dict[str, "object"]:
        """dr_state_export's columns as numpy views (owned by the state until its release)."""
        e = N.dr_export()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_export(self.h, which, C.byref(e)))
        return self._columns(e)

    def export_plan(self, which: int, max_rows: int, max_bytes: int) -> List[int]:
        """dr_state_export_plan: row boundaries of ranges holding at most max_rows rows and at most
        max_bytes bytes in every column (ABI 3)."""
        b = C.POINTER(C.c_int64)()
        n = C.c_int64()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_export_plan(self.h, which, int(max_rows), int(max_bytes),
                                                             C.byref(b), C.byref(n)))
        res = [b[i] for i in range(n.value + 1)]
        self.eng.lib.dr_free(C.cast(b, C.c_void_p))
        return res

    def export_range(self, which: int, lo: int, hi: int) -> Dict[str, "object"]:
        """dr_state_export_range: rows [lo, hi) as columns with offsets rebased to the range, copied
        into numpy arrays (the library's range is released before returning)."""
        e = N.dr_export()
        h = C.c_void_p()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_export_range(self.h, which, int(lo), int(hi), C.byref(h), C.byref(e)))
        try:
            return {k: v.copy() for k, v in self._columns(e).items()}
        finally:
            self.eng.lib.dr_range_release(h)

    def filter(self, program) -> List[int]:
        from .predicates import lower_program
        pred, keep = lower_program(program)
        sel = C.POINTER(C.c_int64)()
        n = C.c_int64()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_filter(self.h, C.byref(pred), C.byref(sel), C.byref(n)))
        res = [sel[i] for i in range(n.value)]
        self.eng.lib.dr_free(C.cast(sel, C.c_void_p))
        return res

    def write_checkpoint_part(self, part: int, parts: int, stats: bool = True, parsed: bool = True,
                              row_group_rows: int = 0, snappy: bool = True, with_adds: bool = False):
        """dr_state_write_checkpoint: part `part` (1-based) of `parts` as Parquet bytes, the file-action
        columns encoded (and SNAPPY-compressed) on the GPU; returns (bytes, rows), or (bytes, rows,
        add rows) with `with_adds`. The bytes are a read-only memoryview of the library's pinned block
        (no copy; released when the view is dropped)."""
        buf = C.POINTER(C.c_uint8)()
        n = C.c_uint64()
        rows = C.c_int64()
        adds = C.c_int64()
        opts = (N.DR_CKPT_STATS if stats else 0) | (N.DR_CKPT_PARSED if parsed else 0) | (N.DR_CKPT_SNAPPY if snappy else 0)
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_write_checkpoint(self.h, int(part), int(parts), opts, int(row_group_rows),
                                                                  C.byref(buf), C.byref(n), C.byref(rows),
                                                                  C.byref(adds)))
        data = _owned_bytes(self.eng.lib, buf, n.value)
        return (data, rows.value, adds.value) if with_adds else (data, rows.value)

    def _take(self, ptr, n) -> List[int]:
        res = [ptr[i] for i in range(n)]
        self.eng.lib.dr_free(C.cast(ptr, C.c_void_p))
        return res

    def scan_order(self) -> List[int]:
        """dr_state_scan_order: live export positions sorted by (modificationTime, path bytes) on the
        GPU (DeltaSourceSnapshot's allFiles.sort, D/files/DeltaSourceSnapshot.scala:53-95)."""
        out = C.POINTER(C.c_int64)()
        n = C.c_int64()
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_scan_order(self.h, C.byref(out), C.byref(n)))
        return self._take(out, n.value)

    def partition_groups(self, rows: Optional[Sequence[int]] = None) -> List[List[int]]:
        """dr_state_partition_groups: `rows` (live export positions; None = all) grouped by the
        table's partition values on the GPU (TahoeFileIndex.listFiles, D/files/TahoeFileIndex.scala:58-81)."""
        order = C.POINTER(C.c_int64)()
        off = C.POINTER(C.c_int64)()
        ng = C.c_int64()
        arr = (C.c_int64 * max(len(rows), 1))(*rows) if rows is not None else None
        with self.eng.lock:
            self.eng.check(self.eng.lib.dr_state_partition_groups(
                self.h, C.cast(arr, C.POINTER(C.c_int64)) if arr is not None else None,
                len(rows) if rows is not None else 0, C.byref(order), C.byref(off), C.byref(ng)))
        nrows = len(rows) if rows is not None else self.counts["num_files"]
        o = self._take(order, nrows)
        g = self._take(off, ng.value + 1)
        return [o[g[k]:g[k + 1]] for k in range(ng.value)]

    def release(self) -> None:
        if self.h:
            with self.eng.lock:
                self.eng.lib.dr_state_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


# ---- retention (DeltaConfigs.TOMBSTONE_RETENTION, D/DeltaConfig.scala:325-331) -----------------
_UNIT_MS = {"millisecond": 1, "milliseconds": 1, "ms": 1, "second": 1000, "seconds": 1000,
            "minute": 60_000, "minutes": 60_000, "hour": 3_600_000, "hours": 3_600_000,
            "day": 86_400_000, "days": 86_400_000, "week": 604_800_000, "weeks": 604_800_000,
            "microsecond": 0.001, "microseconds": 0.001}
DEFAULT_TOMBSTONE_RETENTION = "interval 1 week"


def interval_millis(s: str) -> int:
    """CalendarInterval -> ms (DeltaConfigs.getMilliSeconds); months/years are rejected."""
    t = s.strip().lower()
    if t.startswith("interval"):
        t = t[len("interval"):].strip()
    total = 0.0
    toks = t.split()
    if not toks or len(toks) % 2:
        raise ValueError("invalid interval %r" % s)
    for i in range(0, len(toks), 2):
        unit = toks[i + 1]
        if unit not in _UNIT_MS:
            raise ValueError("unsupported interval unit %r" % unit)
        total += float(toks[i]) * _UNIT_MS[unit]
    return int(total)


def tombstone_retention_millis(metadata: Optional[dict]) -> int:
    conf = (metadata or {}).get("configuration") or {}
    return interval_millis(conf.get("delta.deletedFileRetentionDuration", DEFAULT_TOMBSTONE_RETENTION))


# CalendarInterval parsing (IntervalUtils.safeStringToInterval, as DeltaConfigs.parseCalendarInterval
# reads a table property) and CalendarInterval.toString, for the retention policies that
# DeltaErrors.logFileNotFoundException renders (D/DeltaErrors.scala:451-461; D/DeltaConfig.scala:251-281).
_IV_UNITS = {"year": ("m", 12), "years": ("m", 12), "month": ("m", 1), "months": ("m", 1),
             "week": ("d", 7), "weeks": ("d", 7), "day": ("d", 1), "days": ("d", 1),
             "hour": ("u", 3_600_000_000), "hours": ("u", 3_600_000_000),
             "minute": ("u", 60_000_000), "minutes": ("u", 60_000_000),
             "second": ("u", 1_000_000), "seconds": ("u", 1_000_000),
             "millisecond": ("u", 1000), "milliseconds": ("u", 1000),
             "microsecond": ("u", 1), "microseconds": ("u", 1)}


def calendar_interval(s: str) -> Tuple[int, int, int]:
    """(months, days, microseconds) of an interval string such as "interval 2 weeks"."""
    from decimal import Decimal
    t = s.strip().lower()
    if t.startswith("interval"):
        t = t[len("interval"):].strip()
    toks = t.split()
    if not toks or len(toks) % 2:
        raise ValueError("invalid interval %r" % s)
    acc = {"m": 0, "d": 0, "u": 0}
    for i in range(0, len(toks), 2):
        kind, mul = _IV_UNITS[toks[i + 1]]
        v = Decimal(toks[i]) * mul
        acc[kind] += int(v)
    return acc["m"], acc["d"], acc["u"]


def interval_to_string(months: int, days: int, micros: int) -> str:
    """CalendarInterval.toString (Spark 3.1): "30 days", "1 years 2 months", "7 days 1 hours"."""
    from decimal import Decimal
    if months == 0 and days == 0 and micros == 0:
        return "0 seconds"
    parts = []

    def unit(v, name):
        if v:
            parts.append("%d %s" % (v, name))
    if months:
        unit(int(months / 12), "years")
        unit(months - 12 * int(months / 12), "months")
    unit(days, "days")
    if micros:
        rest = micros
        unit(int(rest / 3_600_000_000), "hours")
        rest -= 3_600_000_000 * int(rest / 3_600_000_000)
        unit(int(rest / 60_000_000), "minutes")
        rest -= 60_000_000 * int(rest / 60_000_000)
        if rest:
            d = (Decimal(rest) / Decimal(1_000_000)).normalize()
            parts.append("%s seconds" % format(d, "f"))
    return " ".join(parts)


def retention_text(metadata: Optional[dict]) -> str:
    """The "(delta.logRetentionDuration=...) and checkpoint retention policy (...)" part of
    logFileNotFoundException for a table's metadata (defaults 30 days / 2 days)."""
    conf = (metadata or {}).get("configuration") or {}
    log_r = interval_to_string(*calendar_interval(conf.get("delta.logRetentionDuration", "interval 30 days")))
    ck_r = interval_to_string(*calendar_interval(conf.get("delta.checkpointRetentionDuration", "interval 2 days")))
    return ("(delta.logRetentionDuration=%s) and checkpoint retention policy "
            "(delta.checkpointRetentionDuration=%s)" % (log_r, ck_r))


# ---- Snapshot / DeltaLog --------------------------------------------------------------------------
class Snapshot:
    def __init__(self, delta_log: "DeltaLog", version: int, state: State, min_file_retention_timestamp: int):
        self.delta_log = delta_log
        self.version = version
        self.state = state
        self.min_file_retention_timestamp = min_file_retention_timestamp
        c = state.counts
        self.num_of_files = c["num_files"]
        self.size_in_bytes = c["size_in_bytes"]
        self.num_of_removes = c["num_removes"]
        self.num_of_metadata = c["num_metadata"]
        self.num_of_protocol = c["num_protocol"]
        self.num_of_set_transactions = c["num_set_transactions"]
        self.protocol = next((a["protocol"] for a in state.nonfile if "protocol" in a), None)
        self.metadata = next((a["metaData"] for a in state.nonfile if "metaData" in a), None)
        self.set_transactions = [a["txn"] for a in state.nonfile if "txn" in a]
        self._all = None
        self._tomb = None

    @property
    def all_files(self) -> List[dict]:
        if self._all is None:
            self._all = self.state.export(N.DR_LIVE)
        return self._all

    @property
    def tombstones(self) -> List[dict]:
        if self._tomb is None:
            self._tomb = self.state.export(N.DR_TOMBSTONES)
        return self._tomb

    @property
    def transactions(self) -> Dict[str, int]:
        return {t["appId"]: t["version"] for t in self.set_transactions}

    def partition_schema(self) -> Dict[str, str]:
        from .predicates import partition_schema
        return partition_schema(self.metadata)

    def _scan_rows(self, filters: Sequence) -> Optional[List[int]]:
        """Live positions kept by the metadata-only conjuncts of `filters` (None: no pruning)."""
        from .predicates import split_metadata_and_data_predicates, build_program
        parts = (self.metadata or {}).get("partitionColumns") or []
        meta_preds = []
        for f in filters:
            meta_preds.extend(split_metadata_and_data_predicates(f, parts)[0])
        if not meta_preds:
            return None
        return self.state.filter(build_program(self.partition_schema(), meta_preds))

    def files_for_scan(self, filters: Sequence) -> List[dict]:
        """PartitionFiltering.filesForScan: metadata-only conjuncts, evaluated on the GPU."""
        sel = self._scan_rows(filters)
        files = self.all_files
        return list(files) if sel is None else [files[i] for i in sel]

    @property
    def checksum_opt(self) -> Optional[bytes]:
        """ReadChecksum.readChecksum (D/Checksum.scala:101-148): the first line of the version's
        `%020d.crc` (FileNames.checksumFile), or None when it is missing or empty."""
        fn = os.path.join(self.delta_log.log_path, "%020d.crc" % self.version)
        try:
            with open(fn, "rb") as f:
                lines = f.read().splitlines()
        except OSError:
            return None  # delta.checksum.error.missing
        return lines[0] if lines and lines[0] else None  # delta.checksum.error.empty

    def validate_checksum(self, corruption_is_fatal: bool = True) -> Optional[str]:
        """ValidateChecksum.validateChecksum (D/Checksum.scala:155-176). With
        spark.databricks.delta.state.corruptionIsFatal (default true) a mismatch raises the
        reference's IllegalStateException; otherwise the mismatch text is returned."""
        line = self.checksum_opt
        if line is None:
            return None
        try:
            mismatch = self.state.check_checksum(line)
        except ValueError:
            return None  # delta.checksum.error.parsing
        if mismatch is not None and corruption_is_fatal:
            raise DeltaError(N.DR_E_CHECKSUM,
                             "The transaction log has failed integrity checks. We recommend you contact "
                             "Databricks support for assistance. To disable this check, set "
                             "spark.databricks.delta.state.corruptionIsFatal to false. Failed verification at "
                             "version %d of:\n%s" % (self.version, mismatch))
        return mismatch

    def list_files(self, partition_filters: Sequence = ()) -> List[Tuple[tuple, List[dict]]]:
        """TahoeFileIndex.listFiles (D/files/TahoeFileIndex.scala:58-81): the pruned files grouped
        by partitionValues; each group is (partition row cast to the partition schema's types,
        [FileStatus {length, modificationTime, path}]) with paths made absolute under the table
        (absolutePath, :86-93). A file lacking a partition column raises KeyError, as
        `partitionValues(p.name)` throws."""
        from urllib.parse import unquote
        from .predicates import cast_partition_value
        schema = self.partition_schema()
        rows = self._scan_rows(partition_filters)
        files = self.all_files
        out = []
        for grp in self.state.partition_groups(rows):  # grouped on the GPU
            pv = files[grp[0]].get("partitionValues") or {}
            row = tuple(cast_partition_value(pv[c], t) for c, t in schema.items())
            stats = []
            for f in (files[i] for i in grp):
                p = unquote(f["path"].split("://", 1)[-1]) if "://" in f["path"] else unquote(f["path"])
                if not (f["path"].startswith("/") or "://" in f["path"] or f["path"].startswith("file:")):
                    p = os.path.join(self.delta_log.data_path, p)
                stats.append({"length": f["size"], "modificationTime": f["modificationTime"], "path": p})
            out.append((row, stats))
        return out

    def initial_files(self, filters: Sequence = ()) -> List[dict]:
        """DeltaSourceSnapshot.initialFiles + iterator (D/files/DeltaSourceSnapshot.scala:53-95):
        allFiles sorted by (modificationTime, path) -- Spark's string order is the UTF-8 byte
        order -- indexed by that order, then the partition-only filters applied (on the GPU, as
        filterFileList with the "add" prefix). Returns IndexedFile records."""
        files = self.all_files
        order = self.state.scan_order()  # sorted on the GPU
        rank = {i: r for r, i in enumerate(order)}
        parts = (self.metadata or {}).get("partitionColumns") or []
        from .predicates import is_partition_only, build_program
        # whole filters, not conjuncts (DeltaTableUtils.isPredicatePartitionColumnsOnly, :46-51)
        preds = [f for f in filters if is_partition_only(f, parts)]
        keep = set(range(len(files)))
        if preds:
            keep = set(self.state.filter(build_program(self.partition_schema(), preds)))
        return [{"version": self.version, "index": rank[i], "add": files[i], "remove": None, "cdc": None,
                 "isLast": False} for i in order if i in keep]

    def release(self) -> None:
        """Frees the resident state now (Snapshot.uncache). Snapshots replaced by `update` are not
        released by it -- a caller may still hold one, as in the reference, where a replaced
        snapshot stays usable -- and free their HBM when they are garbage-collected."""
        self.state.release()


class DeltaLog:
    _cache: Dict[Tuple[str, int], "DeltaLog"] = {}
    _lock = threading.Lock()

    def __init__(self, data_path: str, clock=None, device: int = 0):
        self.data_path = os.path.abspath(data_path)
        self.log_path = os.path.join(self.data_path, "_delta_log")
        self.clock = clock or SystemClock()
        self.engine = Engine.get(device)
        self._snapshot: Optional[Snapshot] = None
        self._lock = threading.RLock()  # deltaLogLock (D/DeltaLog.scala:84)
        self._snapshot = self._build(-1)

    @classmethod
    def for_table(cls, data_path: str, clock=None, device: int = 0) -> "DeltaLog":
        key = (os.path.abspath(data_path), device)
        with cls._lock:
            dl = cls._cache.get(key)
            if dl is None:
                dl = DeltaLog(data_path, clock, device)
                cls._cache[key] = dl
            return dl

    @classmethod
    def clear_cache(cls) -> None:
        """DeltaLog.clearCache: drops the cached logs; their snapshots are freed once unreferenced."""
        with cls._lock:
            for dl in cls._cache.values():
                dl._snapshot = None
            cls._cache.clear()

    @property
    def min_file_retention_timestamp(self) -> int:
        md = self._snapshot.metadata if self._snapshot is not None else None
        return self.clock.get_time_millis() - tombstone_retention_millis(md)

    def _build(self, version: int) -> Snapshot:
        if not os.path.isdir(self.log_path):
            raise DeltaError(3, "No file found in the directory: %s." % self.log_path)
        cutoff = self.min_file_retention_timestamp
        try:
            staged = self.engine.stage_log(self.log_path, version)
        except DeltaError as e:
            # logFileNotFoundException renders the current snapshot's retention policies
            # (SnapshotManagement's `metadata`, D/SnapshotManagement.scala:161-163); the library's
            # listing has no metadata and renders the defaults, as on a first load
            if e.status == 4 and self._snapshot is not None:
                msg = re.sub(r"\(delta\.logRetentionDuration=.*\)$", retention_text(self._snapshot.metadata),
                             str(e))
                raise DeltaError(4, msg) from None
            raise

        try:
            ver, _ = self.engine.log_segment(self.log_path, version)
            state = staged.replay(cutoff)
        finally:
            staged.release()
        return Snapshot(self, ver, state, cutoff)

    @property
    def snapshot(self) -> Snapshot:
        return self._snapshot

    def update(self, incremental: bool = False) -> Snapshot:
        """SnapshotManagement.update (D/SnapshotManagement.scala:286-330). The reference rebuilds
        the snapshot from the new segment; with `incremental` the commits after the current
        version are applied to the resident state instead (dr_state_apply)."""
        with self._lock:
            if incremental and self._snapshot is not None:
                new = self._apply_new_commits()
                if new is None:
                    return self._snapshot
            else:
                new = self._build(-1)
            # replaceSnapshot (D/SnapshotManagement.scala:333-339): the old snapshot's state is
            # freed when its last reference goes (a caller may still be using it)
            self._snapshot = new
            return new

    def _apply_new_commits(self) -> Optional[Snapshot]:
        """The commits after the current version, applied to the resident state; a full rebuild
        (the reference's behaviour) when the tail is not a contiguous run of commits after it, a
        newer checkpoint exists (log cleanup may have removed commits), or the library cannot
        extend the state (DR_E_REBUILD: e.g. a retention cutoff that moved backwards)."""
        cur = self._snapshot
        ver, seg = self.engine.log_segment(self.log_path)
        if ver == cur.version:
            return None
        names = sorted(n for n in os.listdir(self.log_path)
                       if re.fullmatch(r"\d{20}\.json", n) and int(n[:20]) > cur.version)
        vers = [int(n[:20]) for n in names]
        ckpt = max((v for kind, v, _, _ in seg if kind == N.DR_FILE_CHECKPOINT), default=-1)
        if not vers or vers != list(range(cur.version + 1, cur.version + 1 + len(vers))) or ckpt > cur.version \
                or vers[-1] != ver:
            return self._build(-1)
        files = []
        for n in names:
            with open(os.path.join(self.log_path, n), "rb") as f:
                files.append((int(n[:20]), N.DR_FILE_JSON, 0, f.read()))
        cutoff = self.min_file_retention_timestamp
        staged = self.engine.stage_files(files)
        try:
            state = cur.state.apply(staged, cutoff)
        except DeltaError as e:
            if e.status != N.DR_E_REBUILD:
                raise
            return self._build(-1)
        finally:
            staged.release()
        return Snapshot(self, vers[-1], state, cutoff)

    def checkpoint(self, parts: int = 1, device: bool = True) -> dict:
        """Checkpoints.checkpoint (D/Checkpoints.scala:119-141): write the current snapshot's
        checkpoint (multi-part when parts > 1) and `_last_checkpoint` (delta_amd/checkpoint.py):
        Parquet pages encoded on the GPU (device=True) or by Arrow from the device export."""
        from .checkpoint import write_checkpoint, write_checkpoint_device
        with self._lock:
            if device:
                return write_checkpoint_device(self._snapshot, parts=parts)
            return write_checkpoint(self._snapshot, parts=parts)

    def get_changes(self, start_version: int, fail_on_data_loss: bool = False):
        """DeltaLog.getChanges (D/DeltaLog.scala:222-238): (version, [Action.fromJson(line)])
        for every delta file at or after start_version (delta_amd/actions.py)."""
        from .actions import get_changes
        return get_changes(self.log_path, start_version, fail_on_data_loss)

    def get_snapshot_at(self, version: int) -> Snapshot:
        with self._lock:
            if self._snapshot is not None and self._snapshot.version == version:
                return self._snapshot
            return self._build(version)


class InMemoryLogReplay:
    """D/actions/InMemoryLogReplay.scala:35-77 over the GPU engine: `append` buffers each
    version's actions (as their JSON encoding), `checkpoint` replays them on the device and
    returns protocol, metadata, txns, then the live AddFiles and unexpired tombstones sorted by
    path (dataChange=false)."""

    def __init__(self, min_file_retention_timestamp: int, device: int = 0):
        self.min_file_retention_timestamp = int(min_file_retention_timestamp)
        self.engine = Engine.get(device)
        self.current_version = -1
        self._files: List[Tuple[int, int, int, bytes]] = []

    def append(self, version: int, actions: Iterable[dict]) -> None:
        assert self.current_version == -1 or version == self.current_version + 1, (
            "Attempted to replay version %d, but state is at %d" % (version, self.current_version))
        self.current_version = version
        body = "".join(json.dumps(a, separators=(",", ":")) + "\n" for a in actions)
        self._files.append((version, N.DR_FILE_JSON, 0, body.encode()))

    def checkpoint(self) -> List[Tuple[str, dict]]:
        staged = self.engine.stage_files(self._files)
        try:
            st = staged.replay(self.min_file_retention_timestamp, validate=False)
        finally:
            staged.release()
        try:
            out: List[Tuple[str, dict]] = []
            for a in st.nonfile:
                (k, v), = a.items()
                out.append((k, v))
            files = [("add", f) for f in st.export(N.DR_LIVE)] + [("remove", f) for f in st.export(N.DR_TOMBSTONES)]
            files.sort(key=lambda kv: kv[1]["path"])
            return out + files
        finally:
            st.release()
