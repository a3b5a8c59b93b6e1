#!/bin/bash
# 8-wave ring tiles (33/34): kernel tests, isolated tile bench, in-step retune restricted to TILES, step A/B.
# usage: gpurun --timeout 1200 -- bash tools/gpu/ring_check.sh TAG TILES BUDGET
TAG=${1:-x}
TILES=${2:-34}
BUDGET=${3:-500}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "phased or ring_256 or split_k or layer_norm_fused" > gpurun_out/pytest_ring_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_ring_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_ring_$TAG.log
timeout -k 10 300 python tools/tilebench.py --tiles 26,33,34,11 --rounds 3 > gpurun_out/tilebench_$TAG.txt 2>&1 || exit 1
STEPTUNE_ARGS="--only-tiles $TILES" bash tools/gpu/steptune.sh $TAG $BUDGET
