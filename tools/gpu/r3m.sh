#!/bin/bash
TAG=${1:-x}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k "group_norm" > gpurun_out/r3m_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3m_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3m_kern_$TAG.log
OLDLIB=libcsk_prev.so bash tools/gpu/libab.sh $TAG
