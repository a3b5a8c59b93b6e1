#!/bin/bash
# Kernel trace of one timed headline job + per-denoising-step busy/idle analysis.
# usage: gpurun --timeout 900 -- bash tools/gpu/jobtrace.sh TAG [extra bench args]
TAG=${1:-x}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/jt_$TAG -o jt -- python3 $R/bench.py --steps 1 --warmup 1 "$@" > $R/gpurun_out/jt_$TAG.log 2>&1 || exit $?
cd $R && DB=$(ls gpurun_out/jt_$TAG/*/*.db gpurun_out/jt_$TAG/*.db 2>/dev/null | head -1)
python tools/jobgaps.py "$DB" > gpurun_out/jobgaps_$TAG.txt 2>&1
tail -1 gpurun_out/jt_$TAG.log
cat gpurun_out/jobgaps_$TAG.txt
