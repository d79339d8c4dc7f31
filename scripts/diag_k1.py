"""Diagnostic: K1 device walker vs the PERMISSIVE restatement, listing every mismatch."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from delta_amd.delta_log import Engine  # noqa: E402
from tests.test_gpu_edge_cases import _device_lines, _device_view  # noqa: E402
from tests.test_json_lane import corpus, expected, mutate  # noqa: E402

eng = Engine.get(0)
for probe in ([b'\x0b1}1}'], [b'{"a":1}', b'\x0b1}1}', b'{"a":1}'], [b'\x0b'], [b'{"a":\x0b1}']):
    got = _device_lines(eng, probe)
    print("probe", [(l, _device_view(r), expected(l), r["line"]) for l, r in zip(probe, got)])
rng = random.Random(0xDE17B)
base = corpus()
lines = []
while len(lines) < 60000:
    line = mutate(rng, rng.choice(base))
    if b"\n" in line:
        continue
    try:
        line.decode("utf-8")
    except UnicodeDecodeError:
        continue
    lines.append(line)
got = _device_lines(eng, lines)
print("lines", len(lines), "got", len(got))
bad = [(i, l, _device_view(r), expected(l), r["line"] == l) for i, (l, r) in enumerate(zip(lines, got))
       if _device_view(r) != expected(l)]
print("mismatches", len(bad))
for b in bad[:40]:
    print(b)
