#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu4.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu4.log
if [ $rc -ne 0 ]; then exit $rc; fi
export SDAAS_ROOT=$PWD/gpurun_out/sdaas
CSK_AUTOTUNE=1 timeout -k 10 600 python tools/modelbench.py > gpurun_out/modelbench_tuned.log 2>&1 || exit $?
timeout -k 10 300 python tools/modelbench.py > gpurun_out/modelbench_tuned2.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_hip2.log 2>&1
