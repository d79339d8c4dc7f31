# Step time with one stream vs K1 on a second stream (DR_OVERLAP=1), with and without per-kernel events
set -e
O=gpurun_out/overlap
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-timing --steps 20 > $O/single_notiming.json 2> $O/a.err
DR_OVERLAP=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-timing --steps 20 > $O/overlap_notiming.json 2> $O/b.err
DR_OVERLAP=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/overlap_timing.json 2> $O/c.err
for f in $O/*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'])"; done
