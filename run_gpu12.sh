#!/bin/bash
mkdir -p gpurun_out/tune12 && python -m chiaswarm_amd._build || exit 1
export SDAAS_ROOT=$PWD/gpurun_out/tune12
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/pytest_gpu12.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu12.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/gemmprof.py > gpurun_out/gemmprof12.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc12 -o pmc --output-format csv -- python tools/gemmprof.py --shapes 32768x320x320 --tiles 12,18,19 --iters 3 > gpurun_out/pmc12.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d gpurun_out/pmc12b -o pmc --output-format csv -- python tools/gemmprof.py --shapes 32768x320x320 --tiles 12,18,19 --iters 3 > gpurun_out/pmc12b.log 2>&1 || exit $?
CSK_RETUNE=1 CSK_AUTOTUNE=1 timeout -k 10 900 python tools/modelbench.py --out gpurun_out/modelbench12.json > gpurun_out/modelbench12.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench12.log 2>&1
