#!/bin/bash
# Round 4: GEGLU GEMM tiles on the SDXL / SD2.1 GEGLU shapes (isolated, with and without epilogue).
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python tools/tilebench.py --only gemm --gemms "2048,10240,1280:geglu;8192,5120,640:geglu;32768,2560,320:geglu;512,10240,1280:geglu" \
  --tiles 11,15,27,31,32,34,13,20 --splits 1 --probe --rounds 3 > $O/r6q_geglu_$TAG.txt 2>&1 || { tail -20 $O/r6q_geglu_$TAG.txt; exit 1; }
grep -v amdgpu $O/r6q_geglu_$TAG.txt
