#!/bin/bash
# Which GroupNorms still run a statistics pass; then the driver bench on the current tree.
mkdir -p gpurun_out
timeout -k 10 200 python tools/gn_fallbacks.py > gpurun_out/gn_fallbacks_r5c.log 2>&1 || { tail -20 gpurun_out/gn_fallbacks_r5c.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gn_fallbacks_r5c.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r5c.log 2>&1 || { tail -30 gpurun_out/bench_r5c.log; exit 1; }
grep '^{' gpurun_out/bench_r5c.log | cut -c1-300
