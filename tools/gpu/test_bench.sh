#!/bin/bash
# Whole GPU test suite + headline bench.  usage: gpurun -- bash tools/gpu/test_bench.sh TAG
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
