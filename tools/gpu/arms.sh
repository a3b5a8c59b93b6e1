#!/bin/bash
# GPU tests (-k EXPR), interleaved abstep arms of this tree, then a kernel trace of the base arm.
# usage: gpurun --timeout 600 -- bash tools/gpu/arms.sh TAG "pytest -k expression" ARMS
TAG=${1:-x}
K=${2:-"norm"}
ARMS=${3:-base}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/pytest_arms_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_arms_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_arms_$TAG.log
timeout -k 10 300 python tools/abstep.py --arms $ARMS --rounds 5 > gpurun_out/arms_$TAG.log 2>&1 || exit $?
grep median gpurun_out/arms_$TAG.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/profab_${TAG} -o prof -- python3 $GRAFT_REPO_ROOT/tools/abstep.py --arms base --rounds 2 --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/profab_${TAG}.log 2>&1) || exit $?
