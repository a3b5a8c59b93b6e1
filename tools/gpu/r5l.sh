#!/bin/bash
# Channel-blocked GN apply small-grid plan (gcs0 / gcs1) at CFG batch 8 and batch 2; tests first.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "channel_blocked or group_norm" > gpurun_out/gn_tests_r5l.log 2>&1 || { tail -30 gpurun_out/gn_tests_r5l.log; exit 1; }
tail -1 gpurun_out/gn_tests_r5l.log
timeout -k 10 300 python tools/abstep.py --arms gcs0,gcs1 --rounds 5 > gpurun_out/ab_gcs_b8_r5l.log 2>&1 || { tail -20 gpurun_out/ab_gcs_b8_r5l.log; exit 1; }
tail -2 gpurun_out/ab_gcs_b8_r5l.log
timeout -k 10 300 python tools/abstep.py --batch 2 --arms gcs0,gcs1 --rounds 5 > gpurun_out/ab_gcs_b2_r5l.log 2>&1 || { tail -20 gpurun_out/ab_gcs_b2_r5l.log; exit 1; }
tail -2 gpurun_out/ab_gcs_b2_r5l.log
