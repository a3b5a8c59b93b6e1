#!/bin/bash
# Split-K reduce load batching: kernel tests, then step A/B (batch 8 and 2).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "splitk or split_k" > gpurun_out/skr_tests.txt 2>&1 || { tail -30 gpurun_out/skr_tests.txt; exit 1; }
tail -2 gpurun_out/skr_tests.txt
timeout -k 10 400 python tools/abstep.py --arms skr1,skr8,skr4 --rounds 7 --batch 8 > gpurun_out/skr_ab_b8.txt 2>&1
cat gpurun_out/skr_ab_b8.txt
timeout -k 10 400 python tools/abstep.py --arms skr1,skr8,skr4 --rounds 7 --batch 2 > gpurun_out/skr_ab_b2.txt 2>&1
cat gpurun_out/skr_ab_b2.txt
