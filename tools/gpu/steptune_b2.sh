#!/bin/bash
# In-step table tuning of the CFG-batch-2 (batch-1 job) UNet step, then A/B at CFG 2 and CFG 8: shipped vs tuned.
TAG=${1:-stb2}
BUDGET=${2:-720}
mkdir -p gpurun_out /tmp/tn_$TAG
timeout -k 10 $((BUDGET + 200)) python -u tools/steptune.py --batch 2 --budget $BUDGET --out gpurun_out/tune_$TAG.json > gpurun_out/steptune_$TAG.log 2>&1 || { tail -20 gpurun_out/steptune_$TAG.log; exit 1; }
tail -3 gpurun_out/steptune_$TAG.log
cp gpurun_out/tune_$TAG.json /tmp/tn_$TAG/csk_tune.json
for b in 2 8; do
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > gpurun_out/ab_ship_${TAG}_$b.log 2>&1 || exit 1
  SDAAS_ROOT=/tmp/tn_$TAG timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > gpurun_out/ab_new_${TAG}_$b.log 2>&1 || exit 1
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > gpurun_out/ab_ship2_${TAG}_$b.log 2>&1 || exit 1
done
grep median gpurun_out/ab_*_$TAG_*.log
