"""Headline benchmark: Delta snapshot state reconstruction on MI355X (BASELINE.json metric).

One step = one full device replay of the config-3 LogSegment (10M-file checkpoint + 30 JSON
commits with 30% remove/re-add churn and a tombstone-retention cutoff) whose bytes are already
resident in HBM: JSON tokenization (K1), checkpoint page inflate + decode (K2), path hashing and
partition (K3), per-bucket last-writer-wins + retention + compaction + computedState counters
(K4/K6). `value` = log actions replayed per second over all ranks.

Per-kernel truth without taxing the timed steps: an untimed pass (--profile-steps) brackets every
launch with a HIP event pair on its stream (dr_set_timing; one stream, so the kernels add up to the
step) and gives `kernels`; the timed steps then carry an event pair around the longest kernel only
(dr_set_timing_only), whose average launch inside the timed region is `roofline.avg_launch_ms`,
with its algorithmic bytes against the 8 TB/s HBM peak and, when committed
rocprofv3 PMC passes of this command exist (--pmc-dir), its measured HBM traffic. `pipelines`
aggregates K1 (JSON), SNAPPY and K3+K4 (sort + reduce, against SURVEY.md §8d's 69 B/action budget).

Multi-GPU (torchrun, one rank per GPU): the same table is path-hash sharded over the ranks
(delta_amd/sharded.py): each rank stages a contiguous slice of the segment, parses
it, sends each file action to owner(path) with an RCCL all-to-all, reduces its shard and returns
the verdicts. Strong scaling: `value` = table actions per step / max-over-ranks step time.

cpu_baseline: the C++ restatement of the reference replay (oracle/replay_oracle.cpp: 50 hash
partitions, per-partition last-writer-wins table, sort by path) on the SAME full table, on rank 0
at N=1, on the CPUs the process may use (the cgroup quota, 16 on the box), on all affinity CPUs and on one core; its counters and order-free key sums must equal
the GPU's (full-scale parity, `matches_gpu`).
"""
import argparse
import gc
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SORT_REDUCE = ("k_bucket_hist", "k_bucket_offsets", "k_bucket_scatter", "k_bucket_split", "k_bucket_reduce", "k_bucket_verify",
               "k_bucket_reduce64", "k_bucket_exact", "k_sum_stats", "k_survivor_scan", "k_compact2")
SNAPPY = ("k_snap_spec", "k_snap_assume", "k_snap_entries", "k_snap_regions", "k_snap_resolve", "k_snap_count",
          "k_snap_scan", "k_snap_exec", "k_snap_serial")
JSON = ("k_json_index", "k_json_place", "k_json_lines", "k_json_hard")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_table(path, config, scale, seed=None, workers=16):
    """The seeded synthetic table (delta_amd/testing/synth.py), generated once in a child process
    (its multi-part checkpoints are written by forked workers) and cached under the work dir."""
    marker = os.path.join(path, "expected.json")
    if not os.path.exists(marker):
        t = time.time()
        subprocess.run([sys.executable, "-m", "delta_amd.testing.synth", str(config), path, str(scale), str(workers)],
                       cwd=ROOT, check=True, stdout=subprocess.DEVNULL)
        log("generated config %d scale %g in %.1fs" % (config, scale, time.time() - t))
    with open(marker) as f:
        return json.load(f)


def algorithmic_bytes(kernel, plan, counts):
    """Compulsory HBM bytes of one launch of `kernel`: each input it needs read once,
    each output written once. `counts` are the replay's own counters (None for a rank of the library's
    sharded replay, whose reduce-side action count the bench does not see: K3/K4 then go unpriced)."""
    rows = plan["checkpoint_rows"]
    lines = plan.get("json_lines", counts["num_actions"] - rows if counts else 0)
    ch = plan["snappy_chunks"]
    sin, sout = plan["snappy_in_bytes"], plan["snappy_out_bytes"]
    table = {
        "k_json_index": plan["json_bytes"] + 2 * lines,            # bytes in, u16 slot per line
        "k_json_place": 10 * lines,                                # slot in, u64 position out
        "k_json_lines": plan["json_bytes"] + 8 * lines + 50 * lines,  # line bytes + position in, 50 B record out
        "k_page_copy": 2 * plan["copy_bytes"],
        "k_snap_spec": sin + 60 * ch,                              # compressed bytes in, per-chunk state out
        "k_snap_assume": 16 * ch, "k_snap_entries": 16 * ch, "k_snap_count": 8 * ch, "k_snap_scan": 8 * ch,
        # SURVEY.md 8(d)'s compulsory K2 bytes: the compressed pages in, the decompressed pages out (the
        # start bitmaps and chunk entries it also reads, 4 B per 32 and 4 B per 256 compressed bytes,
        # are the decoder's own intermediate and not credited)
        "k_snap_exec": sin + sout,
        "k_pq_data": plan["pages_decompressed_bytes"] + 44 * rows,
        "k_ckpt_assemble": 182 * rows,
    }
    if counts:
        n = counts["num_actions"]
        fa = counts["num_file_actions"]
        surv = counts["num_files"] + counts["num_removes"]
        table.update({
            "k_bucket_hist": 10 * n,                               # kind, flags, key in (r06: path refs by the producers)
            # kind, flags, key in; size or delTs per file action in; 16 B record out
            "k_bucket_scatter": 10 * n + 24 * fa,
            "k_bucket_reduce": 16 * fa + 4 * surv,                 # records in, survivors out (+ verification)
            "k_compact2": 8 * surv,
        })
    return table.get(kernel)


def pmc_traffic(pmc_dir, kernel):
    """Per-launch HBM bytes of `kernel` from committed rocprofv3 --pmc passes (FETCH_SIZE and
    WRITE_SIZE in separate runs of this same bench command). FETCH_SIZE is doubled: on gfx950 it
    tallies 128-B requests at 64 B (MI355X_MICROARCH.md, HBM section; for k_snap_exec's own loads
    checked against TCC_EA0_RDREQ x 128 B, profiles/r06/calib). Only the replay's launches count:
    the dispatches of the grid size that occurs most often (a bench run also decodes export columns
    with the same kernel on other grids; r05's config-4 figure averaged those in and fell below the
    compulsory bytes). Returns None when absent."""
    import csv
    import glob
    if not pmc_dir or not os.path.isdir(pmc_dir):
        return None
    per, grids = {}, {}
    for fn in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if kernel + "(" not in name and not name.endswith(kernel):
                    continue
                c = row.get("Counter_Name")
                v = float(row.get("Counter_Value", 0) or 0)
                g = row.get("Grid_Size")
                d = per.setdefault(c, {}).setdefault(g, {})
                key = (fn, row.get("Dispatch_Id"))
                d[key] = d.get(key, 0.0) + v
                grids.setdefault(g, set()).add(key)
    if "FETCH_SIZE" not in per or "WRITE_SIZE" not in per:
        return None
    g = max(grids, key=lambda x: len(grids[x]))  # the replay's grid
    if g not in per["FETCH_SIZE"] or g not in per["WRITE_SIZE"]:
        return None
    avg = {c: sum(v[g].values()) / len(v[g]) for c, v in per.items() if g in v}
    return int(2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024)  # KiB -> bytes


def run_replay_oracle(log_path, cutoff, threads, record_sums=False):
    exe = os.path.join(ROOT, "oracle", "_build", "replay_oracle")
    r = subprocess.run([exe, log_path, str(cutoff), "--threads", str(threads), "--partitions", "50"]
                       + (["--record-sums"] if record_sums else []), capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        log("cpu baseline failed:", r.stderr[-2000:])
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_budget():
    """(affinity CPUs, cgroup v2 cpu.max quota in CPUs or None): what this process may run on. On the
    GPU box os.cpu_count() shows the whole machine; the affinity mask and the quota are the share."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(per))
    except (OSError, ValueError):
        pass
    return aff, quota


def cpu_baseline(log_path, cutoff, counts, threads, one_core=True, all_cpus=True):
    """oracle/_build/replay_oracle on the same table. `value` / `cores`: the CPUs this
    process may actually use -- the cgroup quota (16 on the GPU box), else the affinity mask -- or
    `threads` when given. Named extras: every CPU of the affinity mask (the box shows its whole
    machine; more threads than the quota only time-slice) and one core. Its counters and order-free
    key sums (incl. the full-record sums) must equal the GPU's."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "replay_oracle")):
        return None
    aff, quota = cpu_budget()
    threads = threads or min(aff, quota or aff)
    res = run_replay_oracle(log_path, cutoff, threads, record_sums="live_record_sum" in counts)
    if res is None:
        return None
    keys = [k for k in ("num_files", "size_in_bytes", "num_removes", "num_file_actions", "live_key_sum",
                        "tomb_key_sum", "live_record_sum", "tomb_record_sum") if k in res and k in counts]
    mism = {k: (res[k], counts[k]) for k in keys if res[k] != counts[k]}
    if mism:
        log("FULL-SCALE PARITY MISMATCH (cpu, gpu):", mism)
    out = {"value": round(res["num_actions"] / res["total_s"], 1), "unit": "actions/s", "cores": threads,
           "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota,
           "kind": "port", "parse_s": res["parse_s"], "replay_s": res["replay_s"], "read_s": res["read_s"],
           "sample": "the full benchmark table (%d actions: %d checkpoint rows + JSON lines), bytes in memory "
                     "before the clock; C++ restatement of the replay (not Spark: no JVM on the box): "
                     "Parquet+SNAPPY and JSON decode, canonicalize, 50 hash partitions, per-partition "
                     "last-writer-wins, retention, sort by path; %d threads = the CPUs this process may "
                     "use (cgroup quota)" % (res["num_actions"], res["checkpoint_rows"], threads),
           "compared": keys, "matches_gpu": not mism, "record_pass_s": res.get("record_s")}
    runs = []
    if all_cpus and aff != threads:
        runs.append(("all_affinity_cpus", aff))
    if one_core:
        runs.append(("one_core", 1))
    for name, t in runs:
        r = run_replay_oracle(log_path, cutoff, t)
        if r:
            out[name] = {"cores": t, "value": round(r["num_actions"] / r["total_s"], 1), "parse_s": r["parse_s"],
                         "replay_s": r["replay_s"]}
    return out


WORKLOAD = {
    3: "config 3: 10M-file checkpoint + 30 JSON commits, %d actions -> %d live files, 30%% remove/re-add churn, "
       "retention cutoff",
    4: "config 4: 100-part checkpoint, %d actions -> %d live files, 4 partition columns; reconstruction step + "
       "4-column partition predicate (k5_filter)",
}


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def measure_stream(eng, table, exp, args):
    """Config 5 (BASELINE.json configs[4]): the streaming tail. A full replay of the 50M-file
    checkpoint is the base; the 10k commits that follow (3 adds + 2 removes each) are each staged
    (file bytes -> HBM) and applied with dr_state_apply, the retention cutoff advancing 30 s per commit
    so tombstones expire along the way. Reports per-commit stage / apply latencies (p50, p99), the
    one-time index build of the first apply, and parity of the final state with a full replay of the
    whole segment (GPU) and with the CPU restatement (key sums)."""
    import torch
    from delta_amd import _native as N
    log_path = os.path.join(table, "_delta_log")
    c0 = exp["min_file_retention_timestamp"]
    step_ms = 30_000
    v0 = exp["version"] - exp["n_deltas"]
    staged = eng.stage_log(log_path, v0)
    t0 = time.perf_counter()
    base = staged.replay(c0)
    torch.cuda.synchronize()
    base_s = time.perf_counter() - t0
    staged.release()
    commits = []
    for v in range(v0 + 1, exp["version"] + 1):
        with open(os.path.join(log_path, "%020d.json" % v), "rb") as f:
            commits.append((v, N.DR_FILE_JSON, 0, f.read()))

    def run(limit, timing):
        cur, stage_ms, apply_ms, kern = base, [], [], {}
        span_ms.clear()
        eng.set_timing(timing)
        # the interpreter's cyclic collector is this harness's, not the library's: paused for the loop
        # (r05's p99 rose 0.052 -> 0.066 ms with p50 and the kernels flat -- host-side jitter), and run
        # between commits, outside the timed calls
        gc.disable()
        for k, c in enumerate(commits[:limit]):
            t1 = time.perf_counter()
            tail = eng.stage_files([c])
            t2 = time.perf_counter()
            nxt = cur.apply(tail, c0 + (k + 1) * step_ms)
            # dr_state_apply returns once the new state's counters are on the host (its readback's
            # completion word): the apply latency a caller sees. The device synchronize follows,
            # untimed, so that every commit starts from an idle device.
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            if timing and k:
                for kn, ms in eng.last_timings().items():
                    if kn == "end":  # the apply's device span: its first kernel's start to its last's end
                        span_ms.append(ms)
                    if kn in ("start", "end") or kn.startswith("stat."):
                        continue
                    kern[kn.split("#")[0]] = kern.get(kn.split("#")[0], 0.0) + ms
            tail.release()
            if cur is not base:
                cur.release()
            cur = nxt
            stage_ms.append((t2 - t1) * 1e3)
            apply_ms.append((t3 - t2) * 1e3)
            if k % 64 == 63:
                gc.collect(0)
        gc.enable()
        eng.set_timing(False)
        return cur, stage_ms, apply_ms, kern

    span_ms = []
    n_timed = min(200, len(commits))
    cur, _, _, kern = run(n_timed, True)  # per-kernel times (events on) over the first commits
    span = list(span_ms)
    cur.release()
    cur, stage_ms, apply_ms, _ = run(len(commits), False)
    first_ms, rest = apply_ms[0], apply_ms[1:]
    tail_actions = cur.counts["num_actions"] - base.counts["num_actions"]
    final_cut = c0 + len(commits) * step_ms
    staged = eng.stage_log(log_path)
    full = staged.replay(final_cut)
    staged.release()
    keys = ("num_files", "size_in_bytes", "num_removes", "num_actions", "num_file_actions", "live_key_sum",
            "tomb_key_sum", "version")
    mism = {k: (cur.counts[k], full.counts[k]) for k in keys if cur.counts[k] != full.counts[k]}
    rec_cur, rec_full = cur.record_sums(), full.record_sums()  # full records of both sides (untimed)
    if rec_cur != rec_full:
        mism["record_sums"] = (rec_cur, rec_full)
    if mism:
        log("STREAM PARITY MISMATCH (applied, full replay):", mism)
    counts = dict(cur.counts, live_record_sum=rec_cur[0], tomb_record_sum=rec_cur[1])
    full.release()
    cur.release()
    base_counts = dict(base.counts)
    base.release()
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline(log_path, final_cut, counts, args.cpu_threads, one_core=False, all_cpus=False)
    if cpu:
        # the reference has no incremental path: every DeltaLog.update() rebuilds the snapshot from
        # its checkpoint + deltas (D/SnapshotManagement.scala:286-330), so its
        # per-commit cost is one full replay of the final segment
        per_commit_s = cpu["value"] and counts["num_actions"] / cpu["value"]
        cpu["full_replay_actions_per_s"] = cpu["value"]
        cpu["per_commit_ms"] = round(per_commit_s * 1e3, 2)
        cpu["value"] = round(tail_actions / len(commits) / per_commit_s, 2)
        cpu["sample"] = ("one full replay of the final segment (%d actions) per update(), the reference's cost per "
                         "commit (no incremental state, D/SnapshotManagement.scala:286-330); value = tail "
                         "actions per second at that rate. " % counts["num_actions"]) + cpu["sample"]
    kernels = {k: round(v / max(1, n_timed - 1), 4) for k, v in sorted(kern.items(), key=lambda x: -x[1])}
    apply_total_s = sum(rest) / 1e3
    return {
        "metric": "log actions replayed/sec + achieved HBM GB/s, 1/2/4/8 GPU, 10M-file table",
        "value": round(tail_actions / (sum(apply_ms) / 1e3), 1), "unit": "actions/s", "n_gpus": 1,
        "steps": len(commits), "warmup": 0, "ms_per_step": round(sum(apply_ms) / len(apply_ms), 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8/int64", "data": "synthetic",
        "config": {"workload": "config 5: streaming tail, %d commits (3 adds + 2 removes) applied one at a time "
                               "to a %d-file state (dr_state_apply, O(tail) path index)"
                               % (len(commits), base_counts["num_files"]),
                   "scale": args.scale, "base_actions": base_counts["num_actions"], "tail_actions": tail_actions,
                   "cutoff_step_ms": step_ms, "parallelism": "single GPU"},
        "stream": {"base_replay_s": round(base_s, 4), "first_apply_ms": round(first_ms, 3),
                   "apply_ms": {"p50": round(_pct(rest, 0.5), 4), "p99": round(_pct(rest, 0.99), 4),
                                "mean": round(sum(rest) / len(rest), 4), "max": round(max(rest), 4)},
                   "stage_ms": {"p50": round(_pct(stage_ms, 0.5), 4), "p99": round(_pct(stage_ms, 0.99), 4)},
                   "stage_plus_apply_ms": {"p50": round(_pct([a + b for a, b in zip(stage_ms[1:], rest)], 0.5), 4),
                                           "p99": round(_pct([a + b for a, b in zip(stage_ms[1:], rest)], 0.99), 4)},
                   "commits_per_s": round(len(rest) / apply_total_s, 1) if rest else None,
                   # the device-side span of an apply (events on its stream, the first 200 commits):
                   # a flat p99 here and a raised host-side p99 place the tail on the host
                   "device_span_ms": {"p50": round(_pct(span, 0.5), 4), "p99": round(_pct(span, 0.99), 4),
                                      "n": len(span)} if span else None,
                   "matches_full_replay": not mism},
        "roofline": {"bound": "hbm", "kernel": next(iter(kernels), None), "achieved": None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": None, "traffic": None,
                     "note": "per-commit kernels touch a few KB: launch/latency-bound, no bandwidth roofline"},
        "cpu_baseline": cpu,
        "kernels_per_commit_ms": kernels,
        "result": {k: counts[k] for k in ("num_files", "num_removes", "size_in_bytes", "live_key_sum", "tomb_key_sum",
                                          "live_record_sum", "tomb_record_sum")},
    }


def measure_checkpoint_write(eng, staged, cutoff, parts):
    """Config 4's multi-part checkpoint write (dr_state_write_checkpoint, file-action pages encoded on
    the GPU, D/Checkpoints.scala:229-365): every part of `parts` written to host memory (no disk; each
    part's bytes dropped after it is counted), after the first call's device export of both sides; the
    whole write's time, bytes and rows, and one part's time for the per-part rate."""
    st = staged.replay(cutoff)
    t_first = time.perf_counter()
    data, rows, adds = st.write_checkpoint_part(1, parts, with_adds=True)  # first: the device export
    first_s = time.perf_counter() - t_first
    total_rows, total_bytes, total_adds = rows, len(data), adds
    part2 = None
    t0 = time.perf_counter()
    for k in range(2, parts + 1):
        tk = time.perf_counter()
        data, rows, adds = st.write_checkpoint_part(k, parts, with_adds=True)
        if k == 2:
            part2 = (time.perf_counter() - tk, rows, len(data))
        total_rows += rows
        total_adds += adds
        total_bytes += len(data)
        del data
    rest_s = time.perf_counter() - t0
    n_live, n_tomb = st.counts["num_files"], st.counts["num_removes"]
    st.release()
    # the reference's check before _last_checkpoint: the parts' adds equal numOfFiles (D/Checkpoints.scala:325-328)
    assert total_adds == n_live and total_rows >= n_live + n_tomb, (total_adds, total_rows, n_live, n_tomb)
    return {"parts": parts, "all_parts_s": round(first_s + rest_s, 3), "first_part_incl_export_s": round(first_s, 3),
            "rows": total_rows, "add_rows": total_adds, "bytes": total_bytes,
            "rows_per_s": round(total_rows / (first_s + rest_s), 1),
            "part_rows": part2[1] if part2 else rows, "part_bytes": part2[2] if part2 else total_bytes,
            "part_s": round(part2[0], 4) if part2 else round(first_s, 4), "codec": "SNAPPY (device)"}


def measure_filter(eng, staged, cutoff, exp, steps):
    """K5 over the reconstructed state: config 4's 4-column conjunction. The first dr_filter builds the
    state's typed partition-value cache (k_pv_extract); later ones only run k_filter_typed."""
    import torch
    from delta_amd.predicates import build_program, partition_schema
    from delta_amd.testing import synth as S
    st = staged.replay(cutoff)
    meta = next(a["metaData"] for a in st.nonfile if "metaData" in a)
    prog = build_program(partition_schema(meta), S.config4_predicate())
    eng.set_timing(True)
    t0 = time.perf_counter()
    sel = st.filter(prog)
    first_s = time.perf_counter() - t0
    first = eng.last_timings()
    ms = {}
    for _ in range(steps):  # per-kernel HIP events (their own pass: the events cost the call time)
        st.filter(prog)
        for k, v in eng.last_timings().items():
            ms[k] = ms.get(k, 0.0) + v / steps
    eng.set_timing(False)
    t0 = time.perf_counter()
    for _ in range(steps):
        st.filter(prog)
    call_s = (time.perf_counter() - t0) / steps
    n = st.counts["num_files"]
    st.release()
    assert len(sel) == exp["selected"], (len(sel), exp["selected"])
    # the dictionary path (k_filter_dict) reads a u16 code per file and column (4 columns: 8 B) and
    # writes one selection bit per file; the typed path (k_filter_leaf) reads p0 date (4 B) + p1 int
    # (4 B) + p2 string (8 B prefix + 4 B length) + p3 boolean (4 B) + 4 null bytes
    kname = next((k for k in ("k_filter_dict", "k_filter_leaf", "k_filter_typed") if k in ms), "k_filter_typed")
    algo = n * (2 * 4) + n // 8 if kname == "k_filter_dict" else n * (4 + 4 + 12 + 4 + 4) + n // 8
    kt = ms.get(kname)
    # SURVEY.md §8(d)'s K5 budget: 4 B per predicate column + 1 B flag out per file (4 columns: 17 B)
    survey = n * (4 * 4 + 1)
    return {"predicate": "p0 >= DATE'2020-03-01' AND p0 < DATE'2020-06-01' AND p1 IN (1..100) AND p2 = 'w17' "
                         "AND p3 = true", "live_files": n, "selected": len(sel),
            "first_call_s": round(first_s, 4), "cache_build_ms": round(first.get("k_pv_extract", 0.0), 4),
            "call_s": round(call_s, 5), "files_per_s": round(n / call_s, 1),
            "roofline": {"bound": "hbm", "kernel": kname, "avg_launch_ms": round(kt, 4) if kt else None,
                         "algo_bytes": algo, "achieved": round(algo / (kt * 1e-3) / 1e9, 1) if kt else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(algo / (kt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if kt else None,
                         "survey_budget_bytes": survey,
                         "survey_frac": round(survey / (kt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if kt else None,
                         "note": "algo_bytes = what this kernel reads and writes (dictionary codes: 2 B per file "
                                 "and column + 1 bit out; typed cache: 28 B/file + 1 bit); survey_* = SURVEY.md "
                                 "8(d)'s 4 B/column + 1 B budget (17 B/file)"},
            "kernels": {k: round(v, 4) for k, v in ms.items()}}


def merge_rank_reports(every):
    """Rank 0's view of an N > 1 run from every rank's {"rank", "roofline", "pipelines"}: the roofline of
    the rank whose dominant kernel takes longest (the step waits for the slowest rank) with each rank's
    kernel, time and fraction listed, and per pipeline the slowest rank's entry with every rank's
    fraction."""
    roofline = None
    rl = [g for g in every if g.get("roofline")]
    if rl:
        worst = max(rl, key=lambda g: g["roofline"]["avg_launch_ms"])
        roofline = dict(worst["roofline"], rank=worst["rank"],
                        per_rank=[{"rank": g["rank"], "kernel": g["roofline"]["kernel"],
                                   "avg_launch_ms": g["roofline"]["avg_launch_ms"], "frac": g["roofline"]["frac"]}
                                  for g in rl],
                        note="the slowest rank's dominant kernel (max avg_launch_ms over ranks); traffic is null: "
                             "the committed PMC passes are single-GPU")
    pipelines = {}
    names = []
    for g in every:
        names += [n for n in (g.get("pipelines") or {}) if n not in names]
    for name in names:
        pr = [(g["rank"], g["pipelines"][name]) for g in every if (g.get("pipelines") or {}).get(name)]
        if pr:
            r_w, worst = max(pr, key=lambda x: x[1]["ms"])
            pipelines[name] = dict(worst, rank=r_w, per_rank_frac=[p["frac"] for _, p in pr])
        else:
            pipelines[name] = None
    return roofline, pipelines


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher around us: start N rank processes of this same command
    through torch.distributed.run (one rank per GPU, rendezvous on 127.0.0.1) and return their exit
    status. This process has not touched the GPU (no HIP call, not even a device count), so it may
    start them; the ranks check the device count themselves and fail loudly when it is short."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: the CPUs this process may use, the cgroup quota; cpu_budget())")
    ap.add_argument("--pmc-dir", default=None,
                    help="rocprofv3 --pmc passes of this build and config (default profiles/r05/pmc/c<config>)")
    ap.add_argument("--driver", choices=("lib", "torch"), default="lib",
                    help="N > 1: the library's own RCCL replay (dr_replay_sharded, what a JNI host calls) or "
                         "delta_amd/sharded.py over torch.distributed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="time the steps without the roofline kernel's events")
    ap.add_argument("--profile-steps", type=int, default=3, help="untimed steps with an event pair on every launch")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="a context option (dr_ctx_set_option, delta_amd/_native.py OPTIONS), e.g. overlap=0")
    ap.add_argument("--workdir", default=os.environ.get("DR_BENCH_DIR", os.path.join(tempfile.gettempdir(), "dr_bench")))
    args = ap.parse_args()
    if args.pmc_dir is None:
        args.pmc_dir = os.path.join(ROOT, "profiles", "r06", "pmc", "c%d" % args.config)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d but WORLD_SIZE=%d: one rank per GPU" % (args.gpus, world))

    import torch
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    backend = None
    if world > 1:
        import torch.distributed as dist
        # DR_BENCH_BACKEND=gloo rehearses the torch driver on a single GPU (host-staged exchange)
        backend = os.environ.get("DR_BENCH_BACKEND", "nccl")
        if backend == "gloo":
            args.driver = "torch"
        ndev = torch.cuda.device_count()
        if backend == "nccl" and ndev < world:
            raise SystemExit("bench.py --gpus %d: only %d GPU(s) visible to rank %d (RCCL needs one GPU per rank)"
                             % (world, ndev, rank))
        local = local % max(ndev, 1)
        torch.cuda.set_device(local)
        if args.driver == "lib" or backend != "nccl":
            # the library driver exchanges over its own RCCL communicator; torch.distributed only
            # carries the communicator id, the barriers and the max-over-ranks time (host, gloo)
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from delta_amd.delta_log import Engine
    from delta_amd.testing import synth as S

    table = os.path.join(args.workdir, "c%d_s%g" % (args.config, args.scale))
    if rank == 0:
        exp = build_table(table, args.config, args.scale)
    if dist:
        dist.barrier()
    exp = build_table(table, args.config, args.scale)
    eng = Engine.get(local)
    for kv in args.option:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    if args.config == 5:
        if world > 1:
            raise SystemExit("config 5 (streaming tail) is a single-GPU workload")
        print(json.dumps(measure_stream(eng, table, exp, args)), flush=True)
        return
    log_path = os.path.join(table, "_delta_log")
    cutoff = exp["min_file_retention_timestamp"]
    t_stage = time.perf_counter()
    if world == 1:
        staged = eng.stage_log(log_path)
        stage_s = time.perf_counter() - t_stage

        def step():
            st = staged.replay(cutoff)
            c = st.counts
            st.release()
            return c, c
    elif args.driver == "lib":
        from delta_amd.sharded import stage_shard
        box = [Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        comm = eng.comm(box[0], world, rank)
        staged = stage_shard(eng, log_path, world, rank)
        stage_s = time.perf_counter() - t_stage

        def step():
            st = comm.replay_sharded(staged, cutoff)
            c = st.counts  # table-wide counters (all-reduced inside the library)
            lc = st.local_counts()  # this rank's own (K3/K4 pricing)
            st.release()
            return c, lc
    else:
        from delta_amd.sharded import Exchange, replay_sharded, stage_shard
        staged = stage_shard(eng, log_path, world, rank)
        stage_s = time.perf_counter() - t_stage
        ex = Exchange()

        def step():
            st = replay_sharded(staged, cutoff, ex)
            c, lc = st.counts, st.local.counts
            st.release()
            return c, lc
    counts = local_counts = None
    eng.set_timing(True)  # the first warm-up counts the SNAPPY elements for the roofline accounting
    for i in range(max(args.warmup, 1)):
        counts, local_counts = step()
        if i == 0:
            eng.set_timing(False)
    for k in ("num_files", "num_removes", "size_in_bytes", "num_actions", "num_file_actions"):
        assert counts[k] == exp[k], (k, counts[k], exp[k])
    plan = staged.plan()  # this rank's slice (roofline accounting is per rank 0's kernels)
    # per-kernel table: an untimed pass with an event pair around every launch (one stream, so the
    # kernels add up to the step); the timed steps then carry events around the longest kernel only
    kern_ms, kern_n, stats = {}, {}, {}
    prof_steps = max(1, args.profile_steps)
    eng.set_timing(True)
    for _ in range(prof_steps):
        step()
        for k, v in eng.last_timings().items():
            if k.startswith("stat."):  # counters of the timed replay (k_bucket_verify's pairs, path bytes)
                stats[k[5:]] = v
                continue
            base = k.split("#")[0]
            kern_ms[base] = kern_ms.get(base, 0.0) + v
            kern_n[base] = kern_n.get(base, 0) + 1
    eng.set_timing(False)
    kern_ms.pop("start", None)
    kern_ms.pop("end", None)
    dom = max(kern_ms, key=kern_ms.get) if kern_ms else None
    eng.set_timing(not args.no_timing and dom is not None, only=dom)
    dom_ms, dom_n = 0.0, 0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for k, v in eng.last_timings().items():
            if k.split("#")[0] == dom:
                dom_ms += v
                dom_n += 1
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        on_dev = backend == "nccl" and args.driver == "torch"
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    eng.set_timing(False)
    total_actions = counts["num_actions"] * args.steps  # table-wide actions per step
    value = total_actions / elapsed
    ms_per_step = elapsed / args.steps * 1000.0
    kernels = {}
    for k, ms in kern_ms.items():
        per_step = ms / prof_steps
        calls = kern_n[k] / prof_steps
        e = {"ms": round(per_step, 4), "launches": calls}
        b = algorithmic_bytes(k, plan, local_counts) if calls == 1 else None
        if b:
            e["algo_bytes"] = b
            e["gbs"] = round(b / (per_step * 1e-3) / 1e9, 1)
        kernels[k] = e
    roofline = None
    rk = dom
    if kernels and dom in kernels and not kernels[dom].get("algo_bytes"):
        # a small table's longest kernel may be one without a byte model (several launches, an
        # unpriced helper): the longest priced kernel stands in, timed by the profiling pass
        priced = [k for k in kernels if kernels[k].get("algo_bytes")]
        if priced:
            rk = max(priced, key=lambda k: kernels[k]["ms"])
    if kernels and rk in kernels:
        e = kernels[rk]
        # the roofline kernel's average launch, measured inside the timed steps (events on its stream)
        live_ms = dom_ms / dom_n if (dom_n and rk == dom) else e["ms"] / max(e["launches"], 1)
        algo = e.get("algo_bytes")
        achieved = round(algo / (live_ms * 1e-3) / 1e9, 1) if algo and live_ms else None
        roofline = {"bound": "hbm", "kernel": rk, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                    # committed PMC passes are of the default single-GPU command
                    "traffic": pmc_traffic(args.pmc_dir, rk) if world == 1 else None,
                    "algo_bytes": algo, "avg_launch_ms": round(live_ms, 4),
                    "launches_timed": dom_n if rk == dom else 0,
                    "kernels_sum_ms": round(sum(x["ms"] for x in kernels.values()), 3)}
        if rk != dom:
            roofline["note"] = "longest kernel %s has no byte model; the longest priced kernel instead" % dom

    def pipeline(names, algo):
        ms = sum(kernels[k]["ms"] for k in names if k in kernels)
        gbs = algo / (ms * 1e-3) / 1e9 if ms else None
        return {"kernels": [k for k in names if k in kernels], "ms": round(ms, 4), "algo_bytes": algo,
                "achieved": round(gbs, 1) if gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None}

    lines = plan["json_lines"]
    pipelines = {
        "json": pipeline(JSON, plan["json_bytes"] + 58 * lines),
        # compulsory SNAPPY traffic: compressed pages in, decompressed pages out
        "snappy": pipeline(SNAPPY, plan["snappy_in_bytes"] + plan["snappy_out_bytes"]),
        # K3 + K4 together against SURVEY.md §8(d)'s headline budget: 32 B/action (sort) + 37 B/action
        # (reduce, retention, compaction) = 69 B/action; at N > 1 per rank, on the actions it reduced
        "sort_reduce": dict(pipeline(SORT_REDUCE, 69 * local_counts["num_actions"]), target_frac=0.5)
        if local_counts else None,
    }
    if local_counts:
        # the same budget without the byte verifier: north_star's sort + reduce is keyed by the path
        # hash alone ((3)-(4): radix sort on (pathHash, version, ordinal), last-writer-wins); comparing
        # each (loser, winner) pair's path bytes is this build's addition for bit-exact sets under a
        # 64-bit collision, priced on its own bytes below. Reported beside sort_reduce, not instead.
        pipelines["sort_reduce_hash_keyed"] = pipeline([k for k in SORT_REDUCE if k != "k_bucket_verify"],
                                                       69 * local_counts["num_actions"])
    if "verify_pairs" in stats and "k_bucket_verify" in kernels:
        # the verifier on its own path bytes: per (loser, winner) pair its 16-byte reference pair and
        # both paths' bytes (the 69 B/action budget above does not model it)
        pipelines["verify"] = dict(pipeline(["k_bucket_verify"], int(16 * stats["verify_pairs"] + stats["verify_path_bytes"])),
                                   pairs=int(stats["verify_pairs"]), path_bytes=int(stats["verify_path_bytes"]))
    if dist:
        # every rank's roofline and pipelines to rank 0: the line reports the slowest rank's (the step
        # waits for it) and lists each rank's
        every = [None] * world
        dist.all_gather_object(every, {"rank": rank, "roofline": roofline, "pipelines": pipelines})
        if rank == 0:
            roofline, pipelines = merge_rank_reports(every)
    if rank != 0:
        return
    if world == 1:
        # full-record checksums of both sides on the device (untimed), for the full-size parity gate
        st = staged.replay(cutoff)
        t_r = time.perf_counter()
        rec = st.record_sums()
        record_s = time.perf_counter() - t_r
        st.release()
        counts = dict(counts, live_record_sum=rec[0], tomb_record_sum=rec[1])
    cpu = None
    if not args.no_cpu_baseline:
        # rank 0, outside the timed region; at N > 1 the other ranks have finished their steps, and the
        # restatement replays the same full table
        cpu = cpu_baseline(log_path, cutoff, counts, args.cpu_threads, one_core=args.config != 4 and world == 1)
    # end to end once: file bytes -> HBM (read + H2D + page planning), replay, allFiles export
    e2e = None
    if world == 1:
        import ctypes as C
        from delta_amd import _native as N
        def export_once():
            # Snapshot.allFiles + tombstones as host columns straight from a replayed state
            # (dr_state_export: each side's columns are extracted on the device and stream to pinned
            # host memory group by group while the later groups are still being extracted)
            t1 = time.perf_counter()
            st = staged.replay(cutoff)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            ex = N.dr_export()
            for which in (N.DR_LIVE, N.DR_TOMBSTONES):
                eng.check(eng.lib.dr_state_export(st.h, which, C.byref(ex)))
            t3 = time.perf_counter()
            st.release()
            return t2 - t1, t3 - t2

        def materialize_once():
            st = staged.replay(cutoff)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            mat_bytes = st.materialize()  # every field of both sides extracted on the device, resident
            t2 = time.perf_counter()
            st.release()
            return t2 - t1, mat_bytes

        def range_export_once():
            # the JNI drop-in's path to rows (jni/DeltaReplayStateRDD.scala): both
            # sides planned at 1M rows / 2^31 - 1 bytes per column, then every range exported to pinned
            # host columns and released, as the RDD's tasks do; twice on one state (the first pass also
            # extracts each side on the device, the second reads the resident columns)
            from delta_amd.delta_log import State
            st = staged.replay(cutoff)
            torch.cuda.synchronize()
            passes, nr, nbytes, nrows = [], 0, 0, 0
            for rep in range(2):
                t1 = time.perf_counter()
                for which in (N.DR_LIVE, N.DR_TOMBSTONES):
                    bounds = st.export_plan(which, 1 << 20, (1 << 31) - 1)
                    for lo, hi in zip(bounds, bounds[1:]):
                        ex, h = N.dr_export(), C.c_void_p()
                        eng.check(eng.lib.dr_state_export_range(st.h, which, lo, hi, C.byref(h), C.byref(ex)))
                        if rep == 0:
                            nr += 1
                            nrows += hi - lo
                            nbytes += sum(v.nbytes for v in State._columns(ex).values())
                        eng.check(eng.lib.dr_range_release(h))
                passes.append(time.perf_counter() - t1)
            st.release()
            return {"ranges": nr, "rows": nrows, "bytes": nbytes, "first_s": round(passes[0], 4),
                    "s": round(passes[1], 4), "gbs": round(nbytes / passes[1] / 1e9, 2),
                    "note": "every dr_state_export_range of both sides at <= 1M rows / 2^31 - 1 B per column "
                            "(plan included), into pinned host columns, released after each; first_s includes "
                            "the device extraction of both sides"}

        rep_s, exp_first = export_once()   # the context's first export pins its host blocks
        rep2, exp_s = export_once()        # a later snapshot's: the context's pinned cache
        mat_s, mat_bytes = materialize_once()
        rng = range_export_once()
        e2e = {"stage_s": round(stage_s, 3), "replay_s": round(rep2, 4),
               "materialize_s": round(mat_s, 4), "materialized_ms": round((rep2 + mat_s) * 1e3, 2),
               "materialized_bytes": mat_bytes, "export_s": round(exp_s, 4),
               "export_s_first_call": round(exp_first, 4),
               "export_beyond_materialize_s": round(exp_s - mat_s, 4),
               "range_export": rng,
               "actions_per_s_incl_staging": round(counts["num_actions"] / (stage_s + rep2), 1),
               "actions_per_s_incl_staging_and_export": round(counts["num_actions"] / (stage_s + rep2 + exp_s), 1),
               "actions_per_s_incl_staging_and_first_export": round(
                   counts["num_actions"] / (stage_s + rep_s + exp_first), 1),
               "note": "materialized_ms = replay + device extraction of every field of both sides (no D2H): the "
                       "resident full-record state; export_s = dr_state_export of both sides from a replayed "
                       "state (extraction + the copy to pinned host columns, overlapped), with the context's "
                       "pinned cache warm (a later snapshot); export_s_first_call pins the blocks"}
    k5 = ckpt = None
    if world == 1 and args.config == 4:
        k5 = measure_filter(eng, staged, cutoff, exp, args.steps)
        ckpt = measure_checkpoint_write(eng, staged, cutoff, parts=100)
    out = {
        "metric": "log actions replayed/sec + achieved HBM GB/s, 1/2/4/8 GPU, 10M-file table",
        "value": round(value, 1), "unit": "actions/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8/int64", "data": "synthetic",
        "config": {"workload": WORKLOAD.get(args.config, "config %d") % (counts["num_actions"], counts["num_files"]),
                   "scale": args.scale, "actions": counts["num_actions"],
                   "json_bytes": exp["json_bytes"], "checkpoint_bytes": exp["checkpoint_bytes"],
                   "parallelism": ("path-hash shards over %d GPUs (%s all-to-all, %s driver)"
                                   % (world, "RCCL" if backend == "nccl" else "gloo rehearsal",
                                      "dr_replay_sharded" if args.driver == "lib" else "torch.distributed"))
                   if world > 1 else "single GPU"},
        "roofline": roofline,
        # the whole step against the HBM roofline: the staged input (JSON + checkpoint bytes, each read
        # once at least) over the step time
        "step_frac": round((exp["json_bytes"] + exp["checkpoint_bytes"]) / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "pipelines": pipelines,
        "cpu_baseline": cpu,
        "end_to_end": e2e,
        "k5_filter": k5,
        "checkpoint_write": ckpt,
        "kernels": kernels,
        "result": dict({k: counts[k] for k in ("num_files", "num_removes", "size_in_bytes", "live_key_sum",
                                               "tomb_key_sum", "live_record_sum", "tomb_record_sum") if k in counts},
                       record_sums_s=round(record_s, 3) if world == 1 else None),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
