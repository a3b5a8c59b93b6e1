#!/bin/bash
# Round 4: the latency-bound mid-size GEMMs (M2048 N1280 K1280: 197 calls per SDXL
# step, 30 per SD2.1 step) over every tile / split, with and without epilogue /
# residual; then the in-step tuner on the SDXL CFG-batch-2 step.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 400 python tools/tilebench.py --only gemm --gemms "2048,1280,1280;8192,640,640;2048,3840,1280;2048,1280,5120" \
  --tiles 11,12,13,14,17,18,19,20,26,27,28,29,33 --splits 1,2,4 --probe --res --rounds 3 > $O/r6j_tiles_$TAG.txt 2>&1 || { tail -20 $O/r6j_tiles_$TAG.txt; exit 1; }
grep -v amdgpu $O/r6j_tiles_$TAG.txt
timeout -k 10 1000 python tools/steptune.py --model sdxl --batch 2 --latent 128 --budget 800 --out $O/tune_step_sdxl_$TAG.json > $O/r6j_steptune_$TAG.log 2>&1 || { tail -20 $O/r6j_steptune_$TAG.log; exit 1; }
tail -30 $O/r6j_steptune_$TAG.log
