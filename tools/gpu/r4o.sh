#!/bin/bash
# In-step tuning with the split-K 16 candidates: 16x16-level convs and the M = 512 / 2048 GEMMs.
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/steptune.py --keys "c:8:16:16:" --budget 300 --out gpurun_out/tune_16_r4o.json > gpurun_out/steptune_16_r4o.log 2>&1 || { tail -20 gpurun_out/steptune_16_r4o.log; exit 1; }
tail -12 gpurun_out/steptune_16_r4o.log
timeout -k 10 700 python -u tools/steptune.py --keys "g:512:" --budget 240 --out gpurun_out/tune_512_r4o.json > gpurun_out/steptune_512_r4o.log 2>&1 || { tail -20 gpurun_out/steptune_512_r4o.log; exit 1; }
tail -12 gpurun_out/steptune_512_r4o.log
