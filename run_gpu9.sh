#!/bin/bash
# correctness of the FAST staging paths + new workflows, then retune + bench
mkdir -p gpurun_out/tune && python -m chiaswarm_amd._build || exit 1
export SDAAS_ROOT=$PWD/gpurun_out/tune
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu9.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu9.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/convprof.py --tiles 1,2,6,11,12,14,15,17 > gpurun_out/convprof9.log 2>&1 || exit $?
CSK_RETUNE=1 CSK_AUTOTUNE=1 timeout -k 10 900 python tools/modelbench.py > gpurun_out/modelbench9.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench9.log 2>&1 || exit $?
timeout -k 10 600 python tools/bench_configs.py --only audioldm,bark,sdxl,esrgan > gpurun_out/configs9.log 2>&1
