#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 600 python tools/opbench.py --out gpurun_out/opbench.json > gpurun_out/opbench.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hip -o hip --output-format csv -- python bench.py --steps 1 --warmup 1 --denoise-steps 10 > gpurun_out/prof_hip.log 2>&1
