#!/bin/bash
# Round 4: 32x32x16 (attn32 1) vs 16x16x32 pipelined (attn32 0) d=64 attention on the small S = 1024 grids.
mkdir -p gpurun_out
for sh in 2,1024,1024,20,64 2,1024,1024,10,64 8,1024,1024,10,64 2,256,256,20,64; do
  for a32 in 1 0; do
    timeout -k 10 60 python tools/attnbench.py --shape $sh --attn32 $a32 --iters 30 2>&1 | grep attn32 || exit 1
  done
done
