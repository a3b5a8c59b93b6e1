#!/bin/bash
# Per-call kernel time of the SD2.1 UNet step at CFG batch 2 (batch-1 jobs) (tools/callprof.py) + short-K GEMM tile probes.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cp_$TAG -o cp -- python3 $R/tools/callprof.py --record /tmp/calls_$TAG.json --batch 2 > $R/gpurun_out/cp_$TAG.log 2>&1 || exit $?
cd $R && python tools/callprof.py --db "$(ls /tmp/cp_$TAG/cp_results.db /tmp/cp_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/calls_$TAG.json --json gpurun_out/callprof_$TAG.json > gpurun_out/callprof_$TAG.txt 2>&1 || { cat gpurun_out/callprof_$TAG.txt; ls -R /tmp/cp_$TAG | head; exit 1; }
head -50 gpurun_out/callprof_$TAG.txt
if [ -n "$TILES" ]; then
  timeout -k 10 400 python tools/tilebench.py --tiles $TILES --only gemm --probe --rounds 3 > gpurun_out/tb_$TAG.txt 2>&1 || exit $?
  cat gpurun_out/tb_$TAG.txt
fi
