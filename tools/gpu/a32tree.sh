#!/bin/bash
# attn32 tree-shaped row max (csk_set_attn32 5): numerics, isolated timing, step A/B.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "attn32_trick or split_kv or spike" > gpurun_out/a32tree_tests.txt 2>&1 || { tail -30 gpurun_out/a32tree_tests.txt; exit 1; }
tail -1 gpurun_out/a32tree_tests.txt
for v in 1 5 1 5; do timeout -k 10 60 python tools/attnbench.py --attn32 $v --iters 40; done > gpurun_out/a32tree_bench.txt 2>&1
cat gpurun_out/a32tree_bench.txt | grep -v amdgpu
timeout -k 10 400 python tools/abstep.py --arms a32t1,a32t5 --rounds 7 --batch 8 2>&1 | grep median
timeout -k 10 400 python tools/abstep.py --arms a32t1,a32t5 --rounds 7 --batch 2 2>&1 | grep median
