#!/bin/bash
# Round 4: halo conv numerics + isolated timing vs the tuned implicit-GEMM conv (+GN apply).
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_conv_halo.py > gpurun_out/r6f_test_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/r6f_test_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/halobench.py --batch 8 > gpurun_out/r6f_halo_b8_$TAG.txt 2>&1 || { tail -20 gpurun_out/r6f_halo_b8_$TAG.txt; exit 1; }
grep -v amdgpu gpurun_out/r6f_halo_b8_$TAG.txt
timeout -k 10 300 python tools/halobench.py --batch 2 > gpurun_out/r6f_halo_b2_$TAG.txt 2>&1 || { tail -20 gpurun_out/r6f_halo_b2_$TAG.txt; exit 1; }
grep -v amdgpu gpurun_out/r6f_halo_b2_$TAG.txt
