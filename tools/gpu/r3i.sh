#!/bin/bash
# Short-KV attention kernel: numerics, isolated timing, step A/B; then batch-2 in-step tuning.
TAG=${1:-x}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k "attention" > gpurun_out/r3i_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3i_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3i_kern_$TAG.log
timeout -k 10 200 python tools/abstep.py --arms xkv2,xkv3 --rounds 7 > gpurun_out/r3i_ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3i_ab_$TAG.txt; exit 1; }
grep median gpurun_out/r3i_ab_$TAG.txt
bash tools/gpu/tune_b2.sh $TAG
