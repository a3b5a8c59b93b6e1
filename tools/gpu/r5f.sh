#!/bin/bash
# Channel-blocked GN apply: block width multiples (gcmN arms), tests first.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "channel_blocked" > gpurun_out/gn_tests_r5f.log 2>&1 || { tail -30 gpurun_out/gn_tests_r5f.log; exit 1; }
tail -1 gpurun_out/gn_tests_r5f.log
timeout -k 10 300 python tools/abstep.py --arms gcm1,gcm2,gcm4,gcm8 --rounds 5 > gpurun_out/ab_gcm_r5f.log 2>&1 || { tail -20 gpurun_out/ab_gcm_r5f.log; exit 1; }
tail -4 gpurun_out/ab_gcm_r5f.log
