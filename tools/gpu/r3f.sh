#!/bin/bash
# Regression check of the current tree: headline bench + per-call step profile.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r3f_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/r3f_bench_$TAG.log; exit 1; }
tail -1 gpurun_out/r3f_bench_$TAG.log
timeout -k 10 200 python tools/abstep.py --arms base --rounds 5 > gpurun_out/r3f_ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3f_ab_$TAG.txt; exit 1; }
grep median gpurun_out/r3f_ab_$TAG.txt
bash tools/gpu/callprof.sh $TAG > /dev/null 2>&1 || exit 1
head -30 gpurun_out/callprof_$TAG.txt
