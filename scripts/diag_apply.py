"""Diagnostic for the incremental apply's counters: the random-commit scenario of
tests/test_gpu_parity.py::test_incremental_apply_random_commits, with the live side's size sum and
row count checked against the state's counters after EVERY apply; repeated, with and without a
warm-up parse before it, to tell a race (first bad version varies) from a data-dependent bug."""
import json
import os
import random
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(lp, compact):
    rng = random.Random(0xC0FFEE)
    os.makedirs(lp, exist_ok=True)
    head = ['{"protocol":{"minReaderVersion":1,"minWriterVersion":2}}',
            '{"metaData":{"id":"t","format":{"provider":"parquet","options":{}},"schemaString":"{}",'
            '"partitionColumns":[],"configuration":{}}}']
    pool = ["f%d.parquet" % i for i in range(400)]
    special = {"f7.parquet": ["/abs/f7.parquet", "file:/abs/f7.parquet", "file:///abs/f7.parquet"],
               "f9.parquet": ["dir/f\\u00e99.parquet", "dir/fé9.parquet"]}
    sep = (",", ":") if compact else (", ", ": ")

    def add(p, v, k):
        return json.dumps({"add": {"path": p, "size": 10 + k, "modificationTime": v, "dataChange": True}},
                          ensure_ascii=False, separators=sep).replace("\\\\u", "\\u")

    def rm(p, ts):
        return json.dumps({"remove": {"path": p, "deletionTimestamp": ts, "dataChange": True}},
                          ensure_ascii=False, separators=sep).replace("\\\\u", "\\u")

    def name(p):
        return rng.choice(special[p]) if p in special else p

    versions = [head + [add(name(p), 0, i) for i, p in enumerate(pool[:150])]]
    for v in range(1, 41):
        lines = []
        for _ in range(rng.randint(1, 12)):
            r = rng.random()
            p = rng.choice(pool)
            if r < 0.35:
                lines.append(add(name(p), v, v))
            elif r < 0.7:
                lines.append(rm(name(p), 1000 * v + rng.randint(0, 999)))
            elif r < 0.8:
                a, b = add(name(p), v, 1), rm(name(p), 1000 * v)
                lines.extend([a, b] if rng.random() < 0.5 else [b, a])
            elif r < 0.87:
                lines.append('{"txn":{"appId":"app%d","version":%d,"lastUpdated":%d}}' % (rng.randint(0, 3), v, v))
            elif r < 0.92:
                lines.append('{"metaData":{"id":"t","format":{"provider":"parquet","options":{}},'
                             '"schemaString":"{}","partitionColumns":[],"configuration":{"v":"%d"}}}' % v)
            else:
                lines.append('{"add":{"path":"broken%d.parquet","size":1' % v)
        versions.append(lines)
    for v, lines in enumerate(versions):
        with open(os.path.join(lp, "%020d.json" % v), "w") as f:
            f.write("\n".join(lines) + "\n")
    return rng


def run(engine, lp, rng_state):
    from delta_amd import _native as N
    rng = random.Random()
    rng.setstate(rng_state)

    def commit(v):
        with open(os.path.join(lp, "%020d.json" % v), "rb") as f:
            return (v, N.DR_FILE_JSON, 0, f.read())

    cut = lambda v: 1000 * v - 5000
    staged = engine.stage_log(lp, 0)
    st = staged.replay(cut(0))
    staged.release()
    states = [st]
    bad = []
    v = 0
    while v < 40:
        k = 2 if rng.random() < 0.2 and v + 2 <= 40 else 1
        tail = engine.stage_files([commit(x) for x in range(v + 1, v + k + 1)])
        nxt = states[-1].apply(tail, cut(v + k))
        tail.release()
        v += k
        states.append(nxt)
        live = nxt.export(0)
        size = sum(r.get("size") or 0 for r in live)
        if nxt.counts["size_in_bytes"] != size or nxt.counts["num_files"] != len(live):
            bad.append((v, k, nxt.counts["size_in_bytes"] - size, nxt.counts["num_files"] - len(live)))
    for s in states:
        s.release()
    return bad


def warm(engine, n):
    from tests.test_json_lane import corpus
    base = [l for l in corpus() if b"\n" not in l]
    lines = []
    while len(lines) < n:
        lines.extend(base)
    body = b"".join(l + b"\n" for l in lines[:n])
    staged = engine.stage_files([(0, 0, 0, body)])
    staged.parse_lines()
    staged.release()


def main():
    import torch  # noqa: F401
    from delta_amd.delta_log import Engine
    engine = Engine.get(0)
    reps = int(os.environ.get("REPS", "4"))
    for compact in (False, True):
        d = tempfile.mkdtemp()
        lp = os.path.join(d, "_delta_log")
        rng = build(lp, compact)
        st0 = rng.getstate()
        for mode in ("cold", "warm"):
            for r in range(reps):
                if mode == "warm":
                    warm(engine, 20000)
                bad = run(engine, lp, st0)
                print("compact=%s %s rep %d: first bad %s (of %d)" % (compact, mode, r, bad[:3], len(bad)), flush=True)
        # the commits around the first bad version of the last run
        if bad:
            v = bad[0][0]
            for x in range(max(1, v - bad[0][1] + 1), v + 1):
                with open(os.path.join(lp, "%020d.json" % x)) as f:
                    print("commit %d:\n%s" % (x, f.read()), flush=True)


if __name__ == "__main__":
    main()
