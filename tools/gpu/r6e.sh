#!/bin/bash
# Round 4: per-call profile of the UNet step with the fused cross-attention block and the halo convs.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && CSK_XATTN=1 CSK_CONV_HALO=1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cp_$TAG -o cp -- python3 $R/tools/callprof.py --record /tmp/calls_$TAG.json > $R/gpurun_out/cp_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/cp_$TAG.log; exit 1; }
cd $R && python tools/callprof.py --db "$(ls /tmp/cp_$TAG/cp_results.db /tmp/cp_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/calls_$TAG.json --json gpurun_out/callprof_$TAG.json > gpurun_out/callprof_$TAG.txt 2>&1 || { cat gpurun_out/callprof_$TAG.txt; exit 1; }
head -45 gpurun_out/callprof_$TAG.txt
grep -E "halo|xattn|finalize" gpurun_out/callprof_$TAG.txt
