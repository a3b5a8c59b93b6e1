#!/bin/bash
# GEMM-kernel iteration: kernel numerics (incl. -k filter), isolated tile sweep, same-box step A/B vs the
# previous library (chiaswarm_amd/lib/ab/libcsk_old.so), per-call profile of the new one.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/gi_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gi_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gi_tests_$TAG.log
if [ -n "$TILES" ]; then
  timeout -k 10 300 python tools/tilebench.py --tiles $TILES --only gemm --rounds 3 > gpurun_out/gi_tb_$TAG.txt 2>&1 || exit 1
  cat gpurun_out/gi_tb_$TAG.txt
fi
OLD=$R/chiaswarm_amd/lib/ab/libcsk_old.so
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/gi_ab_${TAG}_$arm.log 2>&1 || { tail -5 gpurun_out/gi_ab_${TAG}_$arm.log; exit 1; }
  echo "$arm $(grep median gpurun_out/gi_ab_${TAG}_$arm.log)"
done
unset CSK_LIB_PATH CSK_ALLOW_STALE
bash tools/gpu/callprof.sh $TAG > /dev/null 2>&1 || exit 1
head -24 gpurun_out/callprof_$TAG.txt
