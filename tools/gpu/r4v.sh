#!/bin/bash
# Full in-step retune pass on the current kernels (LN merge in the consumer, attn32, CFG-shared prefix).
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/steptune.py --budget 900 --out gpurun_out/tune_full_r4v.json > gpurun_out/steptune_full_r4v.log 2>&1 || { tail -20 gpurun_out/steptune_full_r4v.log; exit 1; }
tail -15 gpurun_out/steptune_full_r4v.log
