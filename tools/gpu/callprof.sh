#!/bin/bash
# Per-call kernel time of one UNet step (tools/callprof.py) under rocprofv3 --kernel-trace.
# usage: MODEL=sd21 BATCH=8 bash tools/gpu/callprof.sh TAG   (MODEL: sd21 | sdxl | controlnet)
TAG=${1:-x}
MODEL=${MODEL:-sd21}
BATCH=${BATCH:-8}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cp_$TAG -o cp -- python3 $R/tools/callprof.py --model $MODEL --batch $BATCH $CPEXTRA --record /tmp/calls_$TAG.json > $O/cp_$TAG.log 2>&1 || { tail -20 $O/cp_$TAG.log; exit 1; }
cd $R && python tools/callprof.py --db "$(ls /tmp/cp_$TAG/cp_results.db /tmp/cp_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/calls_$TAG.json --json $O/callprof_$TAG.json > $O/callprof_$TAG.txt 2>&1 || { cat $O/callprof_$TAG.txt; exit 1; }
head -50 $O/callprof_$TAG.txt
