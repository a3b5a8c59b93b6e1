#!/bin/bash
# Round 5: per-call profiles of the CFG-2 SD2.1 step and the SDXL CFG-2 step (latest tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
bash tools/gpu/callprof_b2.sh r5c > /dev/null || exit 1
head -25 $O/callprof_b2_r5c.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cpx_r5c -o cp -- python3 $R/tools/callprof.py --model sdxl --batch 2 --record /tmp/callsx_r5c.json > $O/cpx_r5c.log 2>&1 || { tail -20 $O/cpx_r5c.log; exit 1; }
cd $R && python tools/callprof.py --db "$(ls /tmp/cpx_r5c/cp_results.db /tmp/cpx_r5c/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/callsx_r5c.json --json $O/callprof_sdxl_r5c.json > $O/callprof_sdxl_r5c.txt 2>&1 || { cat $O/callprof_sdxl_r5c.txt; exit 1; }
head -25 $O/callprof_sdxl_r5c.txt
