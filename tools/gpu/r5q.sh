#!/bin/bash
# Attention tests, batch-1 latency and the headline bench on the current tree.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > gpurun_out/attn_tests_r5q.log 2>&1 || { tail -30 gpurun_out/attn_tests_r5q.log; exit 1; }
tail -1 gpurun_out/attn_tests_r5q.log
timeout -k 10 400 python tools/bench_configs.py --only sd21-b1 --reps 3 > gpurun_out/b1_r5q.log 2>&1 || { tail -20 gpurun_out/b1_r5q.log; exit 1; }
grep '{' gpurun_out/b1_r5q.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r5q.log 2>&1 || { tail -30 gpurun_out/bench_r5q.log; exit 1; }
grep '^{' gpurun_out/bench_r5q.log | cut -c1-200
