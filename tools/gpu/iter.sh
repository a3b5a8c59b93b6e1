#!/bin/bash
# One iteration: kernel tests (-k EXPR), opbench subset (FILTER), UNet step vs the old tree, same box.
# usage: gpurun -- bash tools/gpu/iter.sh TAG "pytest -k expr" "opbench filter"
TAG=${1:-x}
K=${2:-"attention or norm"}
FILT=${3:-attn}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python tools/opbench.py --filter "$FILT" --iters 20 --out gpurun_out/opbench_$TAG.json > gpurun_out/opbench_$TAG.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/opbench_$TAG.log
if [ -d cmp_old ]; then
  timeout -k 10 120 python cmp_old/tools/abstep.py --arms base --rounds 3 > gpurun_out/cmp_old_$TAG.log 2>&1 || exit $?
  grep median gpurun_out/cmp_old_$TAG.log
fi
timeout -k 10 120 python tools/abstep.py --arms base --rounds 3 > gpurun_out/abstep_$TAG.log 2>&1 || exit $?
grep median gpurun_out/abstep_$TAG.log
