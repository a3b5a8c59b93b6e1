#!/bin/bash
# rocprofv3 kernel trace of the headline bench (2 timed jobs) -> gpurun_out/prof_TAG/
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1
