#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -k "canny or fused or persistent" > gpurun_out/pytest_gpu14.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu14.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/phaseprof.py > gpurun_out/phaseprof14.log 2>&1 || exit $?
timeout -k 10 900 python tools/bench_configs.py --only sdxl,controlnet,esrgan,audioldm,bark,sd21-b1 > gpurun_out/configs14.log 2>&1
