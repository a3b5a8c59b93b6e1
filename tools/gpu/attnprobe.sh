#!/bin/bash
# Where the d = 64 pipelined attention spends its time: the production variant vs
# probe builds of the same loop without exp (11), K/V loads (12), PV MFMAs (14), QK MFMAs (18).
TAG=${1:-x}
mkdir -p gpurun_out
for shape in 8,4096,4096,5,64 8,1024,1024,10,64; do
  for v in 0 11 12 14 18 0; do
    timeout -k 10 60 python tools/attnbench.py --variant $v --iters 50 --shape $shape >> gpurun_out/attnprobe_$TAG.txt 2>&1 || exit 1
  done
done
cat gpurun_out/attnprobe_$TAG.txt
