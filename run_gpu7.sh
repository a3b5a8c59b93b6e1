#!/bin/bash
# full GPU test suite + headline bench + kernel-trace profile of the bench
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu7.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu7.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench7.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7 -o bench -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof7.log 2>&1
