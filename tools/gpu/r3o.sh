#!/bin/bash
# Baseline after container re-creation: bench + persistent-tile short-K probe.
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_r3o.log 2>&1 || { tail -20 gpurun_out/bench_r3o.log; exit 1; }
tail -1 gpurun_out/bench_r3o.log
timeout -k 10 300 python tools/tilebench.py --only gemm --tiles 19,20,21,22,23,24,11 --probe --rounds 3 > gpurun_out/tilebench_persist_r3o.txt 2>&1 || { tail -20 gpurun_out/tilebench_persist_r3o.txt; exit 1; }
cat gpurun_out/tilebench_persist_r3o.txt
