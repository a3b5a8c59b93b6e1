#!/bin/bash
# In-step tuning of the 8x8-level conv keys with the split-K 16 candidates.
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/steptune.py --keys "c:8:8:8:" --budget 420 --out gpurun_out/tune_8x8_r4n.json > gpurun_out/steptune_8x8_r4n.log 2>&1 || { tail -20 gpurun_out/steptune_8x8_r4n.log; exit 1; }
tail -8 gpurun_out/steptune_8x8_r4n.log
