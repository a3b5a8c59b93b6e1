#!/bin/bash
# Round 4: in-step tuning of the SDXL 1024-px CFG-batch-2 step (whole-step timing
# per candidate), then SDXL / SD2.1 batch-1 / ControlNet latencies with the result.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_xattn.py > $O/r6o_xt_$TAG.log 2>&1 || { tail -30 $O/r6o_xt_$TAG.log; exit 1; }
tail -1 $O/r6o_xt_$TAG.log
timeout -k 10 150 python tools/xattnbench.py --batch 8 > $O/r6o_xattn_$TAG.txt 2>&1 || { tail -20 $O/r6o_xattn_$TAG.txt; exit 1; }
grep -v amdgpu $O/r6o_xattn_$TAG.txt
timeout -k 10 1000 python tools/steptune.py --model sdxl --batch 2 --latent 128 --budget 780 --iters 4 --out $O/tune_step_sdxl_$TAG.json > $O/r6o_st_$TAG.log 2>&1 || { tail -20 $O/r6o_st_$TAG.log; exit 1; }
grep -E "\->|done|start|budget" $O/r6o_st_$TAG.log
CSK_TUNE_FILE=$O/tune_step_sdxl_$TAG.json timeout -k 10 600 python tools/bench_configs.py --only sdxl,sd21-b1,controlnet --reps 3 > $O/r6o_lat_$TAG.jsonl 2> $O/r6o_err.log || { tail -20 $O/r6o_err.log; exit 1; }
cat $O/r6o_lat_$TAG.jsonl
