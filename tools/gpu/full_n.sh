#!/bin/bash
# GPU tests + smoke + headline bench + kernel trace (profile summary for profiles/)
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 300 python tools/abstep.py --arms base --rounds 5 > gpurun_out/abstep_$TAG.log 2>&1 || exit $?
grep median gpurun_out/abstep_$TAG.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1
if [ -d $GRAFT_REPO_ROOT/cmp_old ]; then
  cd $GRAFT_REPO_ROOT && timeout -k 10 200 python cmp_old/tools/abstep.py --arms base --rounds 5 > gpurun_out/cmp_old_$TAG.log 2>&1 && grep median gpurun_out/cmp_old_$TAG.log
fi
