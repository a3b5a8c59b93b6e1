#!/bin/bash
# 32x32x16 attention kernel: numerics then timing against the pipelined 16x16x32 kernel.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r3w.log 2>&1 || { tail -40 gpurun_out/pytest_attn_r3w.log; exit 1; }
tail -2 gpurun_out/pytest_attn_r3w.log
for sh in 8,4096,4096,5,64 4,4096,4096,5,64 8,1024,1024,10,64 8,256,256,20,64 2,4096,4096,5,64; do
  for v in 0 20 23; do
    timeout -k 10 120 python tools/attnbench.py --shape $sh --variant $v >> gpurun_out/attn32_r3w.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/attn32_r3w.txt
