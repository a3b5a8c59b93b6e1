#!/bin/bash
# Round 4: fused cross-attention sub-block + halo 3x3 conv with fused GroupNorm:
# numerics, then attn32 TRICKS variants, then UNet-step A/B of each knob.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_xattn.py tests/test_conv_halo.py > gpurun_out/r6d_test_$TAG.log 2>&1; rc=$?
tail -30 gpurun_out/r6d_test_$TAG.log | grep -E "passed|failed|Error|error|assert" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 2 3 4; do
  timeout -k 10 60 python tools/attnbench.py --attn32 $v --shape 8,4096,4096,5,64 --iters 50 2>&1 | grep attn32 || exit 1
done
for arm in "CSK_XATTN=0 CSK_CONV_HALO=0" "CSK_XATTN=1 CSK_CONV_HALO=0" "CSK_XATTN=0 CSK_CONV_HALO=1" "CSK_XATTN=1 CSK_CONV_HALO=1"; do
  env $arm timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/r6d_step.log 2>&1 || { tail -8 gpurun_out/r6d_step.log; exit 1; }
  echo "$arm $(grep median gpurun_out/r6d_step.log)"
done
