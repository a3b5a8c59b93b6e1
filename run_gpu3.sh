#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention or group_norm" > gpurun_out/pytest_gpu3.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu3.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/opbench.py --filter attn --out gpurun_out/opbench_attn.json > gpurun_out/opbench_attn.log 2>&1 || exit $?
timeout -k 10 300 python tools/opbench.py --filter groupnorm --out gpurun_out/opbench_gn.json > gpurun_out/opbench_gn.log 2>&1 || exit $?
timeout -k 10 500 python tools/modelbench.py > gpurun_out/modelbench.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unet -o unet --output-format csv -- python tools/modelbench.py --only unet --iters 5 > gpurun_out/prof_unet.log 2>&1
