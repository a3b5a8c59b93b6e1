#!/bin/bash
# Per-call profile of the SD2.1 CFG-batch-2 (batch-1 job) UNet step and a 3-run batch-1 latency sample.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cp_b2_$TAG -o cp -- python3 $R/tools/callprof.py --model sd21 --batch 2 --record /tmp/calls_b2_$TAG.json > $O/cp_b2_$TAG.log 2>&1 || { tail -20 $O/cp_b2_$TAG.log; exit 1; }
cd $R && python tools/callprof.py --db "$(ls /tmp/cp_b2_$TAG/cp_results.db /tmp/cp_b2_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/calls_b2_$TAG.json --json $O/callprof_b2_$TAG.json > $O/callprof_b2_$TAG.txt 2>&1 || { cat $O/callprof_b2_$TAG.txt; exit 1; }
head -50 $O/callprof_b2_$TAG.txt
