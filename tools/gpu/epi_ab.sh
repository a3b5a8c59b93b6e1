#!/bin/bash
# Kernel-library change check: GEMM/conv numerics, same-box step A/B (old lib vs new), per-call profile.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/epi_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/epi_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/epi_tests_$TAG.log
OLD=$R/chiaswarm_amd/lib/ab/libcsk_old.so
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/epiab_${TAG}_$arm.log 2>&1 || exit 1
  echo "$arm $(grep median gpurun_out/epiab_${TAG}_$arm.log)"
done
unset CSK_LIB_PATH CSK_ALLOW_STALE
bash tools/gpu/callprof.sh $TAG > /dev/null 2>&1 || exit 1
head -30 gpurun_out/callprof_$TAG.txt
