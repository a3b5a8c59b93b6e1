#!/bin/bash
# attn32 with the next block's QK^T interleaved into the softmax VALU (variant 35) vs variant 20.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r4g.log 2>&1 || { tail -30 gpurun_out/pytest_attn_r4f.log; exit 1; }
tail -1 gpurun_out/pytest_attn_r4g.log
for sh in 8,4096,4096,5,64 4,4096,4096,5,64 8,1024,1024,10,64; do
  for v in 20 35 20 35; do
    timeout -k 10 60 python tools/attnbench.py --variant $v --iters 50 --shape $sh >> gpurun_out/attn_ilv_r4g.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/attn_ilv_r4g.txt
