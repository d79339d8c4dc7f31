"""Test-only stand-in for the device side of a sharded replay (dr_shard_*), built on the CPU oracle.

It lets the multi-GPU driver (delta_amd/sharded.py) -- plan, exchange of counts / records / path
bytes / verdicts over torch.distributed, counter all-reduce, non-file merge -- run on CPU under
gloo with world_size > 1. The record layout matches DR_SHARD_REC_BYTES; `owner` is a test hash
(the device uses xxh64), which the driver never looks at.
"""
import ctypes as C
import struct
import zlib

from oracle import delta_oracle as O
from delta_amd.sharded import shard_plan

REC = struct.Struct("<QqqIBBH")
assert REC.size == 32


class FakeEng:
    device = 0


def _load_units(log_path, units):
    import pyarrow.parquet as pq
    out = []
    for u in units:
        p = log_path + "/" + u["name"]
        if u["kind"] == 1:
            f = pq.ParquetFile(p)
            hi = f.num_row_groups if u["rg_hi"] < 0 else u["rg_hi"]
            cols = [c for c in O._UNWRAP_ORDER if c in f.schema_arrow.names]
            for g in range(u["rg_lo"], hi):
                for row in f.read_row_group(g, columns=cols).to_pylist():
                    out.append(O.unwrap(row))
        else:
            with open(p, "rb") as fh:
                out.extend(O.read_json_actions(fh.read()))
    return out


class FakeStaged:
    def __init__(self, log_path, world, rank, version):
        self.eng = FakeEng()
        self.version = version
        self.units = [u for u in shard_plan(log_path, world) if u["rank"] == rank]
        self.actions = _load_units(log_path, self.units)


class FakeState:
    def __init__(self, counts, nonfile, live, tomb):
        self.counts = counts
        self.nonfile = nonfile
        self._live, self._tomb = live, tomb

    def export(self, which):
        return list(self._live if which == 0 else self._tomb)

    def set_nonfile_json(self, lines, validate=True):
        """dr_state_set_nonfile_json's reduction (the oracle's merge over the rank-ordered lines)."""
        from delta_amd.sharded import merge_nonfile
        self.nonfile, _ = merge_nonfile([lines], self.counts.get("version", -1), validate)

    def release(self):
        pass


class FakeHandle:
    def __init__(self, staged, world):
        self.st = staged
        self.world = world
        send = [[] for _ in range(world)]
        for i, a in enumerate(staged.actions):
            if a is None or a[0] not in (O.ADD, O.REMOVE):
                continue
            path = O.canonicalize_path(a[1]["path"])
            key = O.replay_key(path)
            send[zlib.crc32(key.encode()) % world].append(i)
        self.order = [i for d in send for i in d]
        self.send_counts = [len(d) for d in send]
        self.send_bytes = [sum(len(self._path(i)) for i in d) for d in send]
        self.owner = {}

    def _path(self, i):
        return O.canonicalize_path(self.st.actions[i][1]["path"]).encode()

    def pack(self, rec_ptr, path_ptr):
        recs, paths = [], []
        for i in self.order:
            kind, act = self.st.actions[i]
            p = self._path(i)
            dt = act.get("deletionTimestamp")
            recs.append(REC.pack(zlib.crc32(p), int(act.get("size") or 0), int(dt or 0), len(p),
                                 1 if kind == O.ADD else 2, 1 if dt is not None else 0, 0))
            paths.append(p)
        r, p = b"".join(recs), b"".join(paths)
        if r:
            C.memmove(rec_ptr, r, len(r))
        if p:
            C.memmove(path_ptr, p, len(p))

    def reduce(self, rec_ptr, n, path_ptr, nbytes, cutoff, verdict_ptr):
        raw = C.string_at(rec_ptr, n * REC.size) if n else b""
        pb = C.string_at(path_ptr, nbytes) if nbytes else b""
        last, off = {}, 0
        recs = []
        for j in range(n):
            key, size, dt, plen, kind, flags, _ = REC.unpack_from(raw, j * REC.size)
            path = pb[off:off + plen].decode()
            off += plen
            recs.append((kind, size, dt if flags else 0))
            last[O.replay_key(path)] = j
        verdict = bytearray(n)
        files = size_sum = removes = 0
        for j in last.values():
            kind, size, dt = recs[j]
            if kind == 1:
                verdict[j] = 1
                files += 1
                size_sum += size
            elif dt > cutoff:
                verdict[j] = 2
                removes += 1
        if n:
            C.memmove(verdict_ptr, bytes(verdict), n)
        self.owner = {"num_files": files, "size_in_bytes": size_sum, "num_removes": removes,
                      "num_file_actions": n}

    def finish(self, verdict_ptr):
        n = len(self.order)
        v = C.string_at(verdict_ptr, n) if n else b""
        live, tomb = [], []
        for j, i in enumerate(self.order):
            kind, act = self.st.actions[i]
            rec = dict(act, path=O.canonicalize_path(act["path"]), dataChange=False)
            if v[j] == 1:
                live.append(rec)
            elif v[j] == 2:
                tomb.append(rec)
        # local non-file winners (the device library's reduce_nonfile without validation)
        r = O.InMemoryLogReplay(0)
        r.append(0, [a for a in self.st.actions if a is not None and a[0] in (O.PROTOCOL, O.METADATA, O.TXN)])
        nonfile = [{k: v2} for k, v2 in r.checkpoint() if k in (O.PROTOCOL, O.METADATA, O.TXN)]
        counts = dict(self.owner, num_actions=len(self.st.actions), malformed_lines=0, live_key_sum=0,
                      tomb_key_sum=0, version=self.st.version)
        return FakeState(counts, nonfile, live, tomb)

    def release(self):
        pass
