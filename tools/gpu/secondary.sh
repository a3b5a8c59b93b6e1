#!/bin/bash
# Secondary BASELINE configs (tools/bench_configs.py) -> gpurun_out/secondary_TAG.jsonl
# usage: bash tools/gpu/secondary.sh TAG [configs] [reps]
TAG=${1:-x}
ONLY=${2:-sd21-b1,sdxl,controlnet,esrgan}
REPS=${3:-5}
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/bench_configs.py --only $ONLY --reps $REPS > gpurun_out/secondary_$TAG.jsonl 2> gpurun_out/secondary_$TAG.err || { tail -20 gpurun_out/secondary_$TAG.err; exit 1; }
cat gpurun_out/secondary_$TAG.jsonl
