#!/bin/bash
# Round 4: key-split attention at S = 1024 on small grids (SDXL 32x32 level B2 H20,
# SD2.1 batch-1 32x32 level B2 H10) and S = 4096 (SDXL 64x64 level B2 H10).
mkdir -p gpurun_out
for sh in 2,1024,1024,20,64 2,1024,1024,10,64 8,1024,1024,10,64 2,4096,4096,10,64; do
  for sp in 1 2 4; do
    timeout -k 10 60 python tools/attnbench.py --shape $sh --split $sp --iters 30 2>&1 | grep attn32 || exit 1
  done
done
