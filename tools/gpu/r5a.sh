#!/bin/bash
# Channel-blocked GN apply (norm.hip gn_apply_cb_kernel): GN tests, then UNet-step A/B off / on.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "group_norm or fused_group" > gpurun_out/gn_tests_r5a.log 2>&1 || { tail -30 gpurun_out/gn_tests_r5a.log; exit 1; }
tail -2 gpurun_out/gn_tests_r5a.log
timeout -k 10 300 python tools/abstep.py --arms gcb0,gcb512,gcb256,gcb1024 --rounds 5 > gpurun_out/ab_gcb_r5a.log 2>&1 || { tail -20 gpurun_out/ab_gcb_r5a.log; exit 1; }
tail -8 gpurun_out/ab_gcb_r5a.log
