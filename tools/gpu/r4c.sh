#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "dup2 or cfg_shared" --timeout 120 --timeout-method thread > gpurun_out/pytest_dup2_r4c.log 2>&1 || { tail -30 gpurun_out/pytest_dup2_r4c.log; exit 1; }
tail -1 gpurun_out/pytest_dup2_r4c.log
timeout -k 10 300 python tools/abstep.py --arms dup0,dup1 --rounds 5 > gpurun_out/abstep_dup_r4c.txt 2>&1 || { tail -20 gpurun_out/abstep_dup_r4c.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/abstep_dup_r4c.txt
