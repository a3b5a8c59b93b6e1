#!/bin/bash
# Round 4: GN apply issues its first x rows before the partials merge (numerics,
# same-box step A/B vs the HEAD library), then the bounds-checking CSK_DEBUG
# build through the whole GPU suite on the current tree.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k "group_norm or gn" > $O/r6n_gn_$TAG.log 2>&1 || { tail -30 $O/r6n_gn_$TAG.log; exit 1; }
tail -1 $O/r6n_gn_$TAG.log
for b in 8 2; do
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > $O/r6n_step.log 2>&1 || { tail $O/r6n_step.log; exit 1; }
  echo "batch $b $arm $(grep median $O/r6n_step.log)"
done
done
unset CSK_LIB_PATH CSK_ALLOW_STALE
CSK_DEBUG=1 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/r6n_debug_suite_$TAG.log 2>&1; rc=$?
tail -5 $O/r6n_debug_suite_$TAG.log
grep -E "FAILED|ERROR|bounds" $O/r6n_debug_suite_$TAG.log | head -20
exit $rc
