#!/bin/bash
# fused GN stats + pipelined attention correctness, op A/B, bench, kernel-trace profile
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu10.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu10.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/opbench.py --out gpurun_out/opbench10.json > gpurun_out/opbench10.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench10.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o bench -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof10.log 2>&1 || exit $?
timeout -k 10 600 python tools/bench_configs.py --only sdxl,esrgan,controlnet,bark,audioldm > gpurun_out/configs10.log 2>&1
