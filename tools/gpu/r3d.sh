#!/bin/bash
TAG=${1:-x}
mkdir -p gpurun_out
bash tools/gpu/attnprobe.sh $TAG || exit 1
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread tests/test_models_gpu.py -k parity > gpurun_out/r3d_models_$TAG.log 2>&1; rc=$?
grep "\[parity\]\|passed\|failed" gpurun_out/r3d_models_$TAG.log
exit $rc
