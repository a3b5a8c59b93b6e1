#!/bin/bash
# 32x32x16 self-attention as the default: numerics, isolated timing, in-step A/B.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r3x.log 2>&1 || { tail -40 gpurun_out/pytest_attn_r3x.log; exit 1; }
tail -2 gpurun_out/pytest_attn_r3x.log
for sh in 8,4096,4096,5,64 4,4096,4096,5,64 8,1024,1024,10,64; do
  for v in 5 20; do
    timeout -k 10 120 python tools/attnbench.py --shape $sh --variant $v >> gpurun_out/attn32_r3x.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/attn32_r3x.txt
timeout -k 10 300 python tools/abstep.py --arms a32off,a32on --rounds 5 > gpurun_out/abstep_attn32_r3x.txt 2>&1 || { tail -20 gpurun_out/abstep_attn32_r3x.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/abstep_attn32_r3x.txt
