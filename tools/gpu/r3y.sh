#!/bin/bash
# Batch-1 latency with the CFG-shared prefix + in-step tuning of the new half-batch (B=1) shapes.
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_configs.py --only sd21-b1 --reps 3 > gpurun_out/b1_before_r3y.log 2>&1 || { tail -20 gpurun_out/b1_before_r3y.log; exit 1; }
grep "{" gpurun_out/b1_before_r3y.log | cut -c1-300
timeout -k 10 700 python -u tools/steptune.py --batch 2 --missing --budget 500 --out gpurun_out/tune_b2dup_r3y.json > gpurun_out/steptune_b2dup_r3y.log 2>&1 || { tail -20 gpurun_out/steptune_b2dup_r3y.log; exit 1; }
tail -12 gpurun_out/steptune_b2dup_r3y.log
