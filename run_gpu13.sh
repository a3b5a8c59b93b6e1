#!/bin/bash
mkdir -p gpurun_out/tune13 && python -m chiaswarm_amd._build || exit 1
export SDAAS_ROOT=$PWD/gpurun_out/tune13
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu13.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu13.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/gemmprof.py > gpurun_out/gemmprof13.log 2>&1 || exit $?
timeout -k 10 300 python tools/opbench.py --filter attn --out gpurun_out/opbench13_attn.json > gpurun_out/opbench13_attn.log 2>&1 || exit $?
CSK_RETUNE=1 CSK_AUTOTUNE=1 timeout -k 10 900 python tools/modelbench.py --out gpurun_out/modelbench13.json > gpurun_out/modelbench13.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench13.log 2>&1
