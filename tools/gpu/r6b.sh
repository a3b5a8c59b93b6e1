#!/bin/bash
# Round 4: attn32 with the row sum on an all-ones PV tile and -mu as one MFMA:
# attention numerics, then attention-only and UNet-step A/B vs the previous library.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_kernels_gpu.py -k "attention" > gpurun_out/r6b_attn_$TAG.log 2>&1 || { tail -30 gpurun_out/r6b_attn_$TAG.log; exit 1; }
tail -1 gpurun_out/r6b_attn_$TAG.log
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  for sh in 8,4096,4096,5,64 8,1024,1024,10,64 2,4096,4096,5,64; do
    timeout -k 10 60 python tools/attnbench.py --shape $sh --iters 50 2>&1 | grep variant | sed "s/^/$arm /" || exit 1
  done
done
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/r6b_step_${TAG}_$arm.log 2>&1 || { tail -5 gpurun_out/r6b_step_${TAG}_$arm.log; exit 1; }
  echo "$arm $(grep median gpurun_out/r6b_step_${TAG}_$arm.log)"
done
