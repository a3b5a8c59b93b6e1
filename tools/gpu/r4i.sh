#!/bin/bash
# attn32 with the conflict-free K/V swizzle: numerics, isolated timing, in-step A/B, PMC of the attention.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r4i.log 2>&1 || { tail -30 gpurun_out/pytest_attn_r4i.log; exit 1; }
tail -1 gpurun_out/pytest_attn_r4i.log
for sh in 8,4096,4096,5,64 4,4096,4096,5,64 8,1024,1024,10,64 8,256,256,20,64; do
  for v in 5 20; do
    timeout -k 10 60 python tools/attnbench.py --variant $v --iters 50 --shape $sh >> gpurun_out/attn_swz_r4i.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/attn_swz_r4i.txt
timeout -k 10 300 python tools/abstep.py --arms a32off,a32on --rounds 5 > gpurun_out/abstep_attn32swz_r4i.txt 2>&1 || { tail -20 gpurun_out/abstep_attn32swz_r4i.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/abstep_attn32swz_r4i.txt
