#!/bin/bash
# Final tree: GPU suite + smoke + headline bench, then the secondary configs (5 reps)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
bash tools/gpu/r5_full.sh $TAG || exit 1
timeout -k 10 700 python tools/bench_configs.py --only sdxl,controlnet,esrgan,sd21-b1 --reps 5 > gpurun_out/secondary_$TAG.jsonl 2> gpurun_out/secondary_$TAG.err || { tail -20 gpurun_out/secondary_$TAG.err; exit 1; }
cat gpurun_out/secondary_$TAG.jsonl
