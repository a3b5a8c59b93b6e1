#!/bin/bash
# Device-resident sampler loop: GPU tests + headline bench + kernel trace of one job.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_loop_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/loop_$TAG.log 2>&1 || { tail -40 gpurun_out/loop_$TAG.log; exit 1; }
tail -3 gpurun_out/loop_$TAG.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
bash tools/gpu/jobtrace.sh $TAG
