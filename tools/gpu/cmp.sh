#!/bin/bash
# Same-box comparison of the UNet step: old tree (cmp_old/) vs this tree, plus tests of this tree.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_cmp.log 2>&1 || { tail -40 gpurun_out/pytest_cmp.log; exit 1; }
tail -1 gpurun_out/pytest_cmp.log
timeout -k 10 300 python cmp_old/tools/abstep.py --arms base --rounds 5 > gpurun_out/cmp_old.log 2>&1 || exit $?
grep median gpurun_out/cmp_old.log
timeout -k 10 300 python tools/abstep.py --arms lnon,lnoff --rounds 5 > gpurun_out/cmp_new.log 2>&1 || exit $?
grep median gpurun_out/cmp_new.log
timeout -k 10 300 python cmp_old/tools/abstep.py --arms base --rounds 5 > gpurun_out/cmp_old2.log 2>&1 || exit $?
grep median gpurun_out/cmp_old2.log
