#!/bin/bash
# Per-call profile of the CFG-batch-2 (batch-1 job) UNet step.
TAG=b2_r4s
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cp_$TAG -o cp -- python3 $R/tools/callprof.py --batch 2 --record /tmp/calls_$TAG.json > $R/gpurun_out/cp_$TAG.log 2>&1 || exit $?
cd $R && python tools/callprof.py --db "$(ls /tmp/cp_$TAG/cp_results.db /tmp/cp_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/calls_$TAG.json --json gpurun_out/callprof_$TAG.json > gpurun_out/callprof_$TAG.txt 2>&1 || { cat gpurun_out/callprof_$TAG.txt; exit 1; }
head -32 gpurun_out/callprof_$TAG.txt
