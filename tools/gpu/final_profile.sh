#!/bin/bash
# Final-tree profiling: kernel tests (incl. the probe-act guard), per-call
# UNet step profile, PMC passes over the UNet step and the VAE decode.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py > $O/r6r_test_$TAG.log 2>&1 || { tail -30 $O/r6r_test_$TAG.log; exit 1; }
tail -1 $O/r6r_test_$TAG.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cp_$TAG -o cp -- python3 $R/tools/callprof.py --record /tmp/calls_$TAG.json > $O/cp_$TAG.log 2>&1 || { tail -20 $O/cp_$TAG.log; exit 1; }
cd $R && python tools/callprof.py --db "$(ls /tmp/cp_$TAG/cp_results.db /tmp/cp_$TAG/*/cp_results.db 2>/dev/null | head -1)" --calls /tmp/calls_$TAG.json --json $O/callprof_$TAG.json > $O/callprof_$TAG.txt 2>&1 || { cat $O/callprof_$TAG.txt; exit 1; }
head -30 $O/callprof_$TAG.txt
bash tools/gpu/pmc_step.sh $TAG || exit 1
head -25 $O/pmcs_${TAG}_1.txt
bash tools/gpu/pmc_decode.sh $TAG || exit 1
