#!/bin/bash
# Round 4: 8-wave xattn workgroup (numerics, probes, step A/B) + the secondary
# model parity tests (SDXL / inpaint / pix2pix / ControlNet / RRDB).
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_xattn.py > gpurun_out/r6h_xt_$TAG.log 2>&1 || { tail -30 gpurun_out/r6h_xt_$TAG.log; exit 1; }
tail -2 gpurun_out/r6h_xt_$TAG.log
timeout -k 10 150 python tools/xattnbench.py --batch 8 > gpurun_out/r6h_xattn_$TAG.txt 2>&1 || { tail -20 gpurun_out/r6h_xattn_$TAG.txt; exit 1; }
grep -v amdgpu gpurun_out/r6h_xattn_$TAG.txt
for arm in "CSK_XATTN_WAVES=4" "CSK_XATTN_WAVES=8"; do
  env $arm timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/r6h_step.log 2>&1 || { tail -8 gpurun_out/r6h_step.log; exit 1; }
  echo "$arm $(grep median gpurun_out/r6h_step.log)"
done
timeout -k 10 600 $PYT -s tests/test_models2_gpu.py > gpurun_out/r6h_m2_$TAG.log 2>&1; rc=$?
grep -E "parity|passed|failed|Error|assert" gpurun_out/r6h_m2_$TAG.log | head -40
exit $rc
