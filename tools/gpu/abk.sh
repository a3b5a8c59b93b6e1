#!/bin/bash
# Same-box A/B with selected GPU tests: pytest -k EXPR, then UNet step old (cmp_old/ = HEAD) vs new, interleaved.
# usage: gpurun --timeout 600 -- bash tools/gpu/abk.sh TAG "pytest -k expression"
TAG=${1:-x}
K=${2:-"norm"}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/pytest_abk_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_abk_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_abk_$TAG.log
timeout -k 10 300 python cmp_old/tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_old_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_new_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python cmp_old/tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_old2_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_new2_$TAG.log 2>&1 || exit $?
grep median gpurun_out/ab_*_$TAG.log
