#!/bin/bash
# Round 4: attention in the cross-attention query projection's epilogue
# (csk_gemm_ln_attn) + xattn on the shared attention header: numerics, then the
# SD2.1 step with the path on / off (CSK_QATTN) at CFG batch 8 and 2, and the
# SDXL / batch-1 latencies.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_qattn.py tests/test_xattn.py > $O/r6s_test_$TAG.log 2>&1 || { tail -40 $O/r6s_test_$TAG.log; exit 1; }
tail -1 $O/r6s_test_$TAG.log
timeout -k 10 150 python tools/xattnbench.py --batch 8 > $O/r6s_xattn_$TAG.txt 2>&1 || { tail -20 $O/r6s_xattn_$TAG.txt; exit 1; }
grep -E "probe  0|probe 15|unfused" $O/r6s_xattn_$TAG.txt
for b in 8 2; do
for arm in 0 1 0 1; do
  CSK_QATTN=$arm timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > $O/r6s_step.log 2>&1 || { tail $O/r6s_step.log; exit 1; }
  echo "batch $b CSK_QATTN=$arm $(grep median $O/r6s_step.log)"
done
done
for arm in 0 1; do
  CSK_QATTN=$arm timeout -k 10 400 python tools/bench_configs.py --only sdxl --reps 3 > $O/r6s_sdxl_$arm.jsonl 2> $O/r6s_err.log || { tail -20 $O/r6s_err.log; exit 1; }
  echo "CSK_QATTN=$arm $(cat $O/r6s_sdxl_$arm.jsonl)"
done
