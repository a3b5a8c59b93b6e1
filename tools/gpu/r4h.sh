#!/bin/bash
# Attention tests after removing the interleave / QB=2 variants, then PMC passes of the current UNet step.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_r4h.log 2>&1 || { tail -30 gpurun_out/pytest_attn_r4h.log; exit 1; }
tail -1 gpurun_out/pytest_attn_r4h.log
bash tools/gpu/pmc_step.sh r4h || exit $?
head -22 gpurun_out/pmcs_r4h_1.txt
