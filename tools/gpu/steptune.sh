#!/bin/bash
# In-step table tuning (tools/steptune.py), then A/B of the UNet step: shipped table vs step-tuned table.
TAG=${1:-st}
BUDGET=${2:-840}
mkdir -p gpurun_out /tmp/tn_$TAG
timeout -k 10 $((BUDGET + 200)) python -u tools/steptune.py $STEPTUNE_ARGS --budget $BUDGET --out gpurun_out/tune_$TAG.json > gpurun_out/steptune_$TAG.log 2>&1 || { tail -20 gpurun_out/steptune_$TAG.log; exit 1; }
tail -3 gpurun_out/steptune_$TAG.log
cp gpurun_out/tune_$TAG.json /tmp/tn_$TAG/csk_tune.json
timeout -k 10 120 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_ship_$TAG.log 2>&1 || exit 1
SDAAS_ROOT=/tmp/tn_$TAG timeout -k 10 120 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_new_$TAG.log 2>&1 || exit 1
timeout -k 10 120 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_ship2_$TAG.log 2>&1 || exit 1
grep median gpurun_out/ab_*_$TAG.log
