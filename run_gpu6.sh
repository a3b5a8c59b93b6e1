#!/bin/bash
mkdir -p gpurun_out && python -m chiaswarm_amd._build || exit 1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_rrdb.py -q -x -k "conv or gemm or rrdb" > gpurun_out/pytest_gpu6.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu6.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/convprof.py > gpurun_out/convprof.log 2>&1 || exit $?
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc1 -o pmc --output-format csv -- python tools/convprof.py --iters 3 > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d gpurun_out/pmc2 -o pmc --output-format csv -- python tools/convprof.py --iters 3 > gpurun_out/pmc2.log 2>&1
