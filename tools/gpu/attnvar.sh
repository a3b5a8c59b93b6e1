#!/bin/bash
# Same-box timing of attention kernel variants on the UNet's self-attention shapes.
TAG=${1:-x}
VARS=${VARS:-0 6 7 9 0}
mkdir -p gpurun_out
for shape in 8,4096,4096,5,64 8,1024,1024,10,64; do
  for v in $VARS; do
    timeout -k 10 60 python tools/attnbench.py --variant $v --iters 50 --shape $shape 2>&1 | grep -v amdgpu.ids >> gpurun_out/attnvar_$TAG.txt || exit 1
  done
done
cat gpurun_out/attnvar_$TAG.txt
