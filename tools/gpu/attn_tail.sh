#!/bin/bash
# Workgroup-count quantisation of the S = 4096 self-attention (1280 WGs at
# B8 H5 = 2.5 rounds of 512 slots) and the GIT GPU test.
set -e
mkdir -p gpurun_out
out=gpurun_out/attn_tail.txt
: > $out
for s in 8,4096,4096,4,64 8,4096,4096,5,64 8,4096,4096,6,64 8,4096,4096,8,64 2,4096,4096,5,64 8,4096,4096,5,64; do
  timeout -k 10 120 python tools/attnbench.py --shape $s --iters 40 >> $out
done
timeout -k 10 120 python tools/attnbench.py --shape 8,4096,4096,5,64 --split 2 --iters 40 >> $out
cat $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_git_caption.py -m gpu \
  > gpurun_out/git_gpu.txt 2>&1
tail -3 gpurun_out/git_gpu.txt
