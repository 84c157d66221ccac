#!/bin/bash
# N>1 bench rehearsal (torchrun, 2 ranks, gloo, virtual devices) + prefill profiles
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
MX_BENCH_VIRTUAL=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r4_bench_n2.json 2> gpurun_out/r4_bench_n2.err
echo "n2 rc=$?"; grep '^{' gpurun_out/r4_bench_n2.json | tail -1 | cut -c1-1200
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_runner_pp -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --tg 8 --no-cpu-baseline --no-dropin --skip-roofline --no-pp2048 > gpurun_out/prof_runner_pp.log 2>&1; echo "prof rc=$?"
