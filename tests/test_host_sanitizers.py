"""The host-only C++ under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer (SURVEY.md
§5: TSAN/ASAN builds of the host library; `make sanitize` builds the same binaries): the LogSegment
listing, the Parquet footer / page planner and small-column host decoder, the host JSON DOM and the host
SNAPPY decoder (tests/native/host_sanitize.cpp, over the reference's golden logs, a synthetic table and
thousands of mutated inputs), and the C++ restatement of the replay (oracle/replay_oracle.cpp) on the
same logs, one thread and four. Any sanitizer report fails the run (-fno-sanitize-recover, TSan's
halt_on_error)."""
import os
import shutil
import subprocess

import pytest

from tests.conftest import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "delta_amd", "csrc")
HOST_SRCS = [os.path.join(CSRC, f) for f in ("log_segment.cpp", "parquet_meta.cpp", "json_host.cpp", "snappy_host.cpp")]
ASAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
TSAN = ["-fsanitize=thread"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
           TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")


def _build(out, srcs, flags):
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-pthread", "-I", os.path.join(ROOT, "include")] + flags +
                       srcs + ["-o", out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    """The golden tables plus a small synthetic table (multi-row-group SNAPPY checkpoint + commits),
    and SNAPPY samples of the kinds the pages hold."""
    import numpy as np
    import pyarrow as pa
    from delta_amd.testing import synth as S
    d = tmp_path_factory.mktemp("san")
    tables = d / "tables"
    shutil.copytree(os.path.join(GOLDEN, "ref"), tables)
    S.build_config(3, str(tables / "synthetic"), scale=0.0005)
    samples = d / "snappy"
    samples.mkdir()
    rng = np.random.default_rng(5)
    payloads = {
        "ints": (np.arange(20000, dtype=np.int64) + 1_700_000_000_000).tobytes(),
        "paths": b"".join(b"p0=2020-01-%02d/p1=%d/part-%05d.snappy.parquet" % (i % 28 + 1, i % 7, i) for i in range(3000)),
        "random": rng.integers(0, 256, 70000, dtype=np.uint8).tobytes(),
    }
    for k, v in payloads.items():
        (samples / k).write_bytes(pa.compress(v, codec="snappy", asbytes=True))
    return str(tables), str(samples)


@pytest.mark.parametrize("kind,threads", [("asan", 1), ("tsan", 4)])
def test_host_code_under_sanitizers(tmp_path, corpus, kind, threads):
    tables, samples = corpus
    exe = str(tmp_path / ("host_" + kind))
    _build(exe, [os.path.join(ROOT, "tests", "native", "host_sanitize.cpp")] + HOST_SRCS, ASAN if kind == "asan" else TSAN)
    r = subprocess.run([exe, tables, str(threads), samples], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout[-2000:] + r.stderr[-4000:]
    assert int(r.stdout.split()[1]) > 1000


@pytest.mark.parametrize("kind,threads", [("asan", 1), ("asan", 4), ("tsan", 4)])
def test_replay_restatement_under_sanitizers(tmp_path, corpus, kind, threads):
    tables, _ = corpus
    exe = str(tmp_path / ("replay_oracle_" + kind))
    _build(exe, [os.path.join(ROOT, "oracle", "replay_oracle.cpp")], ASAN if kind == "asan" else TSAN)
    for name in sorted(os.listdir(tables)):
        lp = os.path.join(tables, name, "_delta_log")
        if not os.path.isdir(lp):
            continue
        r = subprocess.run([exe, lp, "0", "--threads", str(threads), "--partitions", "50", "--record-sums"],
                           capture_output=True, text=True, timeout=600, env=ENV)
        assert r.returncode == 0, name + ": " + r.stderr[-4000:]
