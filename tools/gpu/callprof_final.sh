#!/bin/bash
# Per-call step profiles of the SD2.1 CFG-batch-8 step and the SDXL 1024-px CFG-batch-2 step.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for m in sd21:8 sdxl:2; do
  model=${m%%:*}; b=${m##*:}
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cp_${model}_$TAG -o cp -- python3 $R/tools/callprof.py --model $model --batch $b --record /tmp/calls_${model}_$TAG.json > $O/cp_${model}_$TAG.log 2>&1 || { tail -20 $O/cp_${model}_$TAG.log; exit 1; }
  cd $R && python tools/callprof.py --db "$(ls /tmp/cp_${model}_$TAG/cp_results.db /tmp/cp_${model}_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/calls_${model}_$TAG.json --json $O/callprof_${model}_$TAG.json > $O/callprof_${model}_$TAG.txt 2>&1 || { cat $O/callprof_${model}_$TAG.txt; exit 1; }
  head -12 $O/callprof_${model}_$TAG.txt
done
