#!/bin/bash
# Retune the table keys matching DROP on this box, then A/B the UNet step: shipped table vs retuned table
# (the retuned one loaded as the user table), plus the old tree.  usage: bash tools/gpu/retune_ab.sh TAG DROP [models]
TAG=${1:-x}
DROP=${2:-'^c:'}
MODELS=${3:-sd21}
mkdir -p gpurun_out /tmp/tn_$TAG
export CSK_ENCODER_PROCS=0
timeout -k 10 400 python tools/retune.py --drop "$DROP" --models $MODELS --out gpurun_out/tune_$TAG.json > gpurun_out/retune_$TAG.log 2>&1 || { tail -20 gpurun_out/retune_$TAG.log; exit 1; }
grep -c measured gpurun_out/retune_$TAG.log
cp gpurun_out/tune_$TAG.json /tmp/tn_$TAG/csk_tune.json
if [ -d cmp_old ]; then
  timeout -k 10 120 python cmp_old/tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_old_$TAG.log 2>&1 || exit 1
  grep median gpurun_out/ab_old_$TAG.log
fi
timeout -k 10 120 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_ship_$TAG.log 2>&1 || exit 1
grep median gpurun_out/ab_ship_$TAG.log
SDAAS_ROOT=/tmp/tn_$TAG timeout -k 10 120 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_new_$TAG.log 2>&1 || exit 1
grep median gpurun_out/ab_new_$TAG.log
