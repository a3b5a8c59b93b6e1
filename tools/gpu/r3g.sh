#!/bin/bash
# After reverting the residual-prefetch epilogue: numerics, step A/B of the LN
# row fan-in, headline bench, per-call profile.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_kernels_gpu.py -k "layer_norm or row_fanin or gemm or conv" > gpurun_out/r3g_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3g_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3g_kern_$TAG.log
timeout -k 10 300 python tools/abstep.py --arms rf0,rf1 --rounds 7 > gpurun_out/r3g_ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3g_ab_$TAG.txt; exit 1; }
grep median gpurun_out/r3g_ab_$TAG.txt
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r3g_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/r3g_bench_$TAG.log; exit 1; }
tail -1 gpurun_out/r3g_bench_$TAG.log
bash tools/gpu/callprof.sh $TAG > /dev/null 2>&1 || exit 1
head -24 gpurun_out/callprof_$TAG.txt
