"""bench.py's N > 1 line: every rank's roofline and K3/K4 pricing reach rank 0 (merge_rank_reports, CPU),
and a two-rank gloo rehearsal on one GPU prints roofline, pipelines.sort_reduce and cpu_baseline
(GPU). The driver's 8-GPU run prints the same keys through the library's RCCL driver."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rank(r, dom_ms, sr_ms):
    return {"rank": r,
            "roofline": {"bound": "hbm", "kernel": "k_snap_exec", "achieved": 1000.0 / dom_ms, "peak": 8000.0,
                         "unit": "GB/s", "frac": 0.125 / dom_ms, "traffic": None, "algo_bytes": 10 ** 9,
                         "avg_launch_ms": dom_ms, "launches_timed": 3, "kernels_sum_ms": 5.0},
            "pipelines": {"json": {"ms": 1.0, "frac": 0.1},
                          "sort_reduce": {"ms": sr_ms, "frac": 0.2 / sr_ms, "target_frac": 0.5}}}


def test_merge_rank_reports_takes_the_slowest_rank():
    from bench import merge_rank_reports
    roof, pipes = merge_rank_reports([_rank(0, 1.0, 0.5), _rank(1, 1.5, 0.4), _rank(2, 1.2, 0.7)])
    assert roof["rank"] == 1 and roof["avg_launch_ms"] == 1.5
    assert [p["rank"] for p in roof["per_rank"]] == [0, 1, 2]
    assert pipes["sort_reduce"]["rank"] == 2 and pipes["sort_reduce"]["ms"] == 0.7
    assert len(pipes["sort_reduce"]["per_rank_frac"]) == 3
    assert pipes["json"]["frac"] == 0.1


def test_merge_rank_reports_keeps_missing_pipelines_null():
    from bench import merge_rank_reports
    a, b = _rank(0, 1.0, 0.5), _rank(1, 1.0, 0.5)
    a["pipelines"]["sort_reduce"] = None
    b["pipelines"]["sort_reduce"] = None
    _, pipes = merge_rank_reports([a, b])
    assert pipes["sort_reduce"] is None


@pytest.mark.gpu
def test_two_rank_gloo_rehearsal_line(tmp_path):
    """`bench.py --gpus 2` with DR_BENCH_BACKEND=gloo on one GPU (torch driver, host-staged exchange):
    the line carries the metric with the per-rank roofline, K3/K4 pricing and the CPU baseline."""
    env = dict(os.environ, DR_BENCH_BACKEND="gloo", DR_BENCH_DIR=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29541", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--scale", "0.02", "--profile-steps", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["roofline"] and line["roofline"]["frac"] and len(line["roofline"]["per_rank"]) == 2
    sr = line["pipelines"]["sort_reduce"]
    assert sr and sr["frac"] and len(sr["per_rank_frac"]) == 2
    hk = line["pipelines"]["sort_reduce_hash_keyed"]  # the same budget without the byte verifier
    assert hk and hk["frac"] and len(hk["per_rank_frac"]) == 2
    cpu = line["cpu_baseline"]
    assert cpu and cpu["value"] > 0 and cpu["matches_gpu"]
