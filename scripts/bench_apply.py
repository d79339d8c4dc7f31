"""Incremental tail apply latency (the config-5 shape on the config-3 table):
the resident state of the 10M-file table is extended by K commits of 3 adds + 2 removes each, one
dr_state_apply per commit; prints one JSON line with the per-commit latency p50 / p99 (ms), the
full rebuild time it replaces and the final counters, checked against the expected arithmetic."""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def commit_lines(v, k):
    """Commit v: 3 new adds; removes of 2 of the previous commit's adds (k = commit ordinal)."""
    lines = ['{"commitInfo":{"timestamp":%d,"operation":"WRITE"}}' % (1800000000000 + v)]
    for j in range(3):
        lines.append('{"add":{"path":"p0=2021-01-01/p1=%d/part-inc-%08d-%d.snappy.parquet","partitionValues":'
                     '{"p0":"2021-01-01","p1":"%d"},"size":%d,"modificationTime":%d,"dataChange":true}}'
                     % (k % 1000, k, j, k % 1000, 1000 + j, 1800000000000 + v))
    if k:
        for j in range(2):
            lines.append('{"remove":{"path":"p0=2021-01-01/p1=%d/part-inc-%08d-%d.snappy.parquet",'
                         '"deletionTimestamp":%d,"dataChange":true}}' % ((k - 1) % 1000, k - 1, j, 1800000000000 + v))
    return ("\n".join(lines) + "\n").encode()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--commits", type=int, default=200)
    ap.add_argument("--workdir", default=os.environ.get("DR_BENCH_DIR", os.path.join(tempfile.gettempdir(), "dr_bench")))
    args = ap.parse_args()
    import bench
    from delta_amd import _native as N
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S
    table = os.path.join(args.workdir, "c3_s%g" % args.scale)
    exp = bench.build_table(table, 3, args.scale, S.BASE_SEED + 3)
    eng = Engine.get(0)
    lp = os.path.join(table, "_delta_log")
    cutoff = exp["min_file_retention_timestamp"]
    staged = eng.stage_log(lp)
    state = staged.replay(cutoff)
    t0 = time.perf_counter()
    for _ in range(3):
        state.release()
        state = staged.replay(cutoff)
    rebuild_ms = (time.perf_counter() - t0) / 3 * 1e3
    staged.release()
    v0 = state.counts["version"]
    lat = []
    for k in range(args.commits):
        v = v0 + 1 + k
        tail = eng.stage_files([(v, N.DR_FILE_JSON, 0, commit_lines(v, k))])
        t = time.perf_counter()
        nxt = state.apply(tail, cutoff)
        lat.append((time.perf_counter() - t) * 1e3)
        tail.release()
        state.release()
        state = nxt
    c = state.counts
    K = args.commits
    ok = (c["num_files"] == exp["num_files"] + 3 * K - 2 * (K - 1)
          and c["num_removes"] == exp["num_removes"] + 2 * (K - 1) and c["version"] == v0 + K)
    lat.sort()
    print(json.dumps({"metric": "incremental tail apply latency (3 adds + 2 removes per commit)",
                      "p50_ms": round(lat[len(lat) // 2], 3), "p99_ms": round(lat[min(len(lat) - 1, int(0.99 * len(lat)))], 3),
                      "commits": K, "base_files": exp["num_files"], "full_rebuild_ms": round(rebuild_ms, 3),
                      "counts_ok": ok, "num_files": c["num_files"], "num_removes": c["num_removes"]}), flush=True)
    state.release()


if __name__ == "__main__":
    main()
