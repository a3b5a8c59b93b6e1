#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_i.log 2>&1 || { tail -40 gpurun_out/pytest_i.log; exit 1; }
tail -2 gpurun_out/pytest_i.log
timeout -k 10 400 python tools/abstep.py --arms lnon,lnoff --rounds 5 > gpurun_out/abstep_i.log 2>&1 || exit $?
cat gpurun_out/abstep_i.log | grep median
