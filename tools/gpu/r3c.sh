#!/bin/bash
# Round-3 check: GEMM kernel numerics (incl. B-stationary tiles) + tile sweep,
# fp32-twin model parity, then the CSK_DEBUG build over every kernel test.
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_kernels_gpu.py -k "gemm or tile or conv or group_norm or layer_norm or bstat" > gpurun_out/r3c_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3c_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3c_kern_$TAG.log
timeout -k 10 300 python tools/tilebench.py --tiles ${TILES:-19,20,40,41} --only gemm --rounds 3 > gpurun_out/r3c_tb_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3c_tb_$TAG.txt; exit 1; }
cat gpurun_out/r3c_tb_$TAG.txt
timeout -k 10 400 $PYT tests/test_models_gpu.py -v > gpurun_out/r3c_models_$TAG.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|rel_err" gpurun_out/r3c_models_$TAG.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CSK_DEBUG=1 timeout -k 10 500 $PYT tests/test_kernels_gpu.py tests/test_loop_gpu.py > gpurun_out/r3c_debug_$TAG.log 2>&1 || { tail -40 gpurun_out/r3c_debug_$TAG.log; exit 1; }
tail -2 gpurun_out/r3c_debug_$TAG.log
