#!/bin/bash
# rocprofv3 kernel trace of tools/abstep.py arms (one arm per process) -> gpurun_out/profab_TAG_ARM/
TAG=${1:-x}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for ARM in "$@"; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/profab_${TAG}_$ARM -o prof -- python3 $GRAFT_REPO_ROOT/tools/abstep.py --arms $ARM --rounds 2 --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/profab_${TAG}_$ARM.log 2>&1) || exit $?
  grep median $GRAFT_REPO_ROOT/gpurun_out/profab_${TAG}_$ARM.log
done
