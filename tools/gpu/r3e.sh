#!/bin/bash
# LN row-statistics fan-in: numerics, same-box step A/B; attention variant timings.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_kernels_gpu.py -k "layer_norm or row_fanin or gemm_epilogue or debug" > gpurun_out/r3e_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3e_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3e_kern_$TAG.log
timeout -k 10 300 python tools/abstep.py --arms rf0,rf1 --rounds 7 > gpurun_out/r3e_ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3e_ab_$TAG.txt; exit 1; }
grep median gpurun_out/r3e_ab_$TAG.txt
VARS="0 6 7 9 0" bash tools/gpu/attnvar.sh $TAG
