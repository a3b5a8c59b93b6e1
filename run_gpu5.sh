#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/pytest_gpu5.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu5.log
if [ $rc -ne 0 ]; then exit $rc; fi
export SDAAS_ROOT=$PWD/gpurun_out/sdaas5
CSK_RETUNE=1 CSK_AUTOTUNE=1 timeout -k 10 900 python tools/modelbench.py > gpurun_out/modelbench5_tune.log 2>&1 || exit $?
timeout -k 10 300 python tools/modelbench.py > gpurun_out/modelbench5.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_hip5.log 2>&1
