#!/bin/bash
# Same-box A/B vs the pre-round library, then numerics of the GEMM paths and the headline bench.
TAG=${1:-x}
mkdir -p gpurun_out
bash tools/gpu/libab.sh $TAG || exit 1
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_kernels_gpu.py -k "layer_norm or gemm or conv or debug" > gpurun_out/r3h_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3h_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3h_kern_$TAG.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r3h_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/r3h_bench_$TAG.log; exit 1; }
grep metric gpurun_out/r3h_bench_$TAG.log | cut -c1-330
