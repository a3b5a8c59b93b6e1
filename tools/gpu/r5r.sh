#!/bin/bash
# In-step tuning of the CFG-batch-2 32x32 conv shapes (all tiles, split 16 now a candidate), then A/B at batch 2.
mkdir -p gpurun_out /tmp/tn_r5r
timeout -k 10 560 python -u tools/steptune.py --batch 2 --all-tiles --keys "c:2:32:32:" --budget 300 --out gpurun_out/tune_b2_32x32_r5r.json > gpurun_out/steptune_b2_32x32_r5r.log 2>&1 || { tail -20 gpurun_out/steptune_b2_32x32_r5r.log; exit 1; }
tail -8 gpurun_out/steptune_b2_32x32_r5r.log
cp gpurun_out/tune_b2_32x32_r5r.json /tmp/tn_r5r/csk_tune.json
for arm in ship new ship new; do
  if [ $arm = new ]; then export SDAAS_ROOT=/tmp/tn_r5r; else unset SDAAS_ROOT; fi
  timeout -k 10 150 python tools/abstep.py --batch 2 --arms base --rounds 3 > gpurun_out/ab_${arm}_r5r.log 2>&1 || exit 1
  echo "$arm $(grep median gpurun_out/ab_${arm}_r5r.log)"
done
timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_b8_r5r.log 2>&1 && echo "b8 $(grep median gpurun_out/ab_b8_r5r.log)"
