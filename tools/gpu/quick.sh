#!/bin/bash
# Quick GPU iteration: selected kernel tests (-k EXPR), headline bench, job phase timings.
# usage: gpurun --timeout 900 -- bash tools/gpu/quick.sh TAG "pytest -k expression"
TAG=${1:-x}
K=${2:-"norm"}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/pytest_quick_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_quick_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_quick_$TAG.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
if [ -n "$PHASE" ]; then timeout -k 10 300 python tools/phaseprof.py jobs > gpurun_out/phasejobs_$TAG.log 2>&1 || exit $?; fi
