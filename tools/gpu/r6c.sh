#!/bin/bash
# Round 4: fused cross-attention sub-block (xattn.hip) numerics + UNet-step A/B
# (CSK_XATTN=0/1), and the attn32 TRICKS variants (csk_set_attn32 1..4).
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_xattn.py tests/test_kernels_gpu.py -k "xattn or attention or transformer" > gpurun_out/r6c_test_$TAG.log 2>&1 || { tail -40 gpurun_out/r6c_test_$TAG.log; exit 1; }
tail -1 gpurun_out/r6c_test_$TAG.log
for v in 1 2 3 4 1 2 3 4; do
  for sh in 8,4096,4096,5,64 8,1024,1024,10,64; do
    timeout -k 10 60 python tools/attnbench.py --attn32 $v --shape $sh --iters 50 2>&1 | grep attn32 || exit 1
  done
done
for arm in 0 1 0 1; do
  CSK_XATTN=$arm timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/r6c_step_${TAG}_$arm.log 2>&1 || { tail -5 gpurun_out/r6c_step_${TAG}_$arm.log; exit 1; }
  echo "xattn=$arm $(grep median gpurun_out/r6c_step_${TAG}_$arm.log)"
done
