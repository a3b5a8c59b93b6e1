#!/bin/bash
# Split-KV attention for small grids: numerics, timing vs unsplit, batch-1 latency.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r4t.log 2>&1 || { tail -30 gpurun_out/pytest_attn_r4t.log; exit 1; }
tail -1 gpurun_out/pytest_attn_r4t.log
for sh in 2,4096,4096,5,64 1,4096,4096,5,64 2,1024,1024,10,64; do
  for w in 0 512; do
    CSK_ATTN_SPLIT_WG=$w timeout -k 10 60 python tools/attnbench.py --variant 0 --iters 50 --shape $sh | grep -v amdgpu | sed "s/^/splitwg=$w /" >> gpurun_out/attn_split_r4t.txt || exit 1
  done
done
cat gpurun_out/attn_split_r4t.txt
for w in 0 512; do
  CSK_ATTN_SPLIT_WG=$w timeout -k 10 200 python tools/bench_configs.py --only sd21-b1 --reps 3 > gpurun_out/b1_split${w}_r4t.log 2>&1 || exit 1
  echo "splitwg=$w $(grep '{' gpurun_out/b1_split${w}_r4t.log | cut -c1-200)"
done
