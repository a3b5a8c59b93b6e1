#!/bin/bash
# Attention/LN tests, then cold-cache retune of the SD2.1 table + A/B (shipped vs retuned table).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn or layer_norm" --timeout 200 --timeout-method thread > gpurun_out/pytest_cold.log 2>&1 || { tail -40 gpurun_out/pytest_cold.log; exit 1; }
tail -1 gpurun_out/pytest_cold.log
CSK_TUNE_COLD=1 bash tools/gpu/retune_ab.sh ${1:-cold} "${2:-^[gc]:}" sd21
