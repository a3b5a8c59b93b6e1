#!/bin/bash
# Round 4: SDXL 1024-px batch-1 work: latency, per-call profile of the CFG-batch-2
# step, isolated autotune of the shapes the shipped table lacks, latency again.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 400 python tools/bench_configs.py --only sdxl --reps 3 > $O/r6i_sdxl_before_$TAG.jsonl 2> $O/r6i_err.log || { tail -20 $O/r6i_err.log; exit 1; }
cat $O/r6i_sdxl_before_$TAG.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cpx_$TAG -o cp -- python3 $R/tools/callprof.py --model sdxl --batch 2 --record /tmp/callsx_$TAG.json > $O/r6i_cp.log 2>&1 || { tail -20 $O/r6i_cp.log; exit 1; }
cd $R && python tools/callprof.py --db "$(ls /tmp/cpx_$TAG/cp_results.db /tmp/cpx_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/callsx_$TAG.json --json $O/callprof_sdxl_$TAG.json > $O/callprof_sdxl_$TAG.txt 2>&1 || { cat $O/callprof_sdxl_$TAG.txt; exit 1; }
head -40 $O/callprof_sdxl_$TAG.txt
timeout -k 10 600 python tools/retune.py --models sdxl --out $O/tune_sdxl_$TAG.json > $O/r6i_retune_$TAG.log 2>&1 || { tail -20 $O/r6i_retune_$TAG.log; exit 1; }
grep -c measured $O/r6i_retune_$TAG.log
CSK_TUNE_FILE=$O/tune_sdxl_$TAG.json timeout -k 10 400 python tools/bench_configs.py --only sdxl --reps 3 > $O/r6i_sdxl_after_$TAG.jsonl 2> $O/r6i_err.log || { tail -20 $O/r6i_err.log; exit 1; }
cat $O/r6i_sdxl_after_$TAG.jsonl
