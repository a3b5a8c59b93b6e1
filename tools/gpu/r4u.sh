#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "attention or txt2img or loop" --timeout 200 --timeout-method thread > gpurun_out/pytest_attn_r4u.log 2>&1 || { tail -30 gpurun_out/pytest_attn_r4u.log; exit 1; }
tail -1 gpurun_out/pytest_attn_r4u.log
