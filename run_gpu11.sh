#!/bin/bash
# persistent-kernel correctness, retune with the new tiles, op A/B + bench
mkdir -p gpurun_out/tune11 && python -m chiaswarm_amd._build || exit 1
export SDAAS_ROOT=$PWD/gpurun_out/tune11
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/pytest_gpu11.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu11.log
if [ $rc -ne 0 ]; then exit $rc; fi
CSK_RETUNE=1 CSK_AUTOTUNE=1 timeout -k 10 900 python tools/modelbench.py --out gpurun_out/modelbench11.json > gpurun_out/modelbench11.log 2>&1 || exit $?
timeout -k 10 300 python tools/opbench.py --filter gemm --out gpurun_out/opbench11.json > gpurun_out/opbench11.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench11.log 2>&1
