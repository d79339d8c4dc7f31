# smoke(), then a 2-rank bench rehearsal on the one GPU (gloo exchange, the N>1 code path)
set -e
mkdir -p gpurun_out/reh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/reh/smoke.log 2>&1
DR_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --scale 0.25 > gpurun_out/reh/n2.json 2> gpurun_out/reh/n2.err
tail -1 gpurun_out/reh/smoke.log
tail -1 gpurun_out/reh/n2.json | cut -c1-600
