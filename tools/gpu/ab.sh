#!/bin/bash
# Same-box A/B: kernel/model GPU tests of this tree, then the UNet step of cmp_old/ (HEAD) vs this tree, then bench.
# usage: gpurun --timeout 900 -- bash tools/gpu/ab.sh TAG
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_ab_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_ab_$TAG.log
timeout -k 10 300 python cmp_old/tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_old_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_new_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python cmp_old/tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_old2_$TAG.log 2>&1 || exit $?
grep median gpurun_out/ab_*_$TAG.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
