#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 900 python -m pytest tests/test_workflows_gpu.py tests/test_kernels_gpu.py -q -x > gpurun_out/pytest_gpu8.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu8.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_configs.py --only audioldm,bark,sd21-b1 > gpurun_out/configs8.log 2>&1
