#!/bin/bash
# Large-map GN finalize: numerics + VAE decode / text encode timing, old library vs new (same box).
TAG=${1:-x}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k "group_norm" > gpurun_out/r3k_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3k_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3k_kern_$TAG.log
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 120 python tools/decodeprof.py --iters 5 > gpurun_out/r3k_dec_${TAG}_$arm.log 2>&1 || { tail -5 gpurun_out/r3k_dec_${TAG}_$arm.log; exit 1; }
  echo "$arm $(grep ' ms' gpurun_out/r3k_dec_${TAG}_$arm.log | tr '\n' ' ')"
done
