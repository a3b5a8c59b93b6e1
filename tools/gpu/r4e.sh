#!/bin/bash
# Where attn32 spends its time: production kernel vs probe builds (no exp / no K/V loads / no PV / no QK MFMAs).
mkdir -p gpurun_out
for sh in 8,4096,4096,5,64 8,1024,1024,10,64; do
  for v in 20 31 32 34 38 20; do
    timeout -k 10 60 python tools/attnbench.py --variant $v --iters 50 --shape $sh >> gpurun_out/attn32probe_r4e.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/attn32probe_r4e.txt
