#!/bin/bash
# In-step tuning of the CFG-batch-2 (one image) SD2.1 UNet step shapes + batch-1 latency before/after.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_configs.py --only sd21-b1 --reps 3 > gpurun_out/tb2_before_$TAG.log 2>&1 || { tail -20 gpurun_out/tb2_before_$TAG.log; exit 1; }
grep "{" gpurun_out/tb2_before_$TAG.log | cut -c1-300
timeout -k 10 900 python -u tools/steptune.py --batch 2 --budget 780 --out gpurun_out/tune_b2_$TAG.json > gpurun_out/tb2_tune_$TAG.log 2>&1 || { tail -20 gpurun_out/tb2_tune_$TAG.log; exit 1; }
tail -5 gpurun_out/tb2_tune_$TAG.log
