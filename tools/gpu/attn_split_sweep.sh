#!/bin/bash
mkdir -p gpurun_out
for sh in 2,4096,4096,5,64 1,4096,4096,5,64; do
  for sp in 1 2 3 4 6 8; do
    timeout -k 10 60 python tools/attnbench.py --shape $sh --split $sp --iters 30 2>&1 | grep attn32 || exit 1
  done
done
