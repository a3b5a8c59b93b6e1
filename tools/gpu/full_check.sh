#!/bin/bash
# Full GPU check on a gpurun box: kernel/model tests, smoke, headline bench, kernel trace.
# usage: gpurun --timeout 1200 -- bash tools/gpu/full_check.sh TAG
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1
