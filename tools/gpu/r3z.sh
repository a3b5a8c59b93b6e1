#!/bin/bash
# LN row statistics merged in the consumer GEMM: numerics (every tile, both paths), model parity, step A/B.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "layer_norm or gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest_ln_r3z.log 2>&1 || { tail -40 gpurun_out/pytest_ln_r3z.log; exit 1; }
tail -2 gpurun_out/pytest_ln_r3z.log
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q -k "parity or cfg_shared" --timeout 200 --timeout-method thread -s > gpurun_out/pytest_parity_r3z.log 2>&1 || { tail -40 gpurun_out/pytest_parity_r3z.log; exit 1; }
grep -E "parity\]|passed|failed" gpurun_out/pytest_parity_r3z.log
timeout -k 10 300 python tools/abstep.py --arms lnk0,lnk1 --rounds 5 > gpurun_out/abstep_lnk_r3z.txt 2>&1 || { tail -20 gpurun_out/abstep_lnk_r3z.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/abstep_lnk_r3z.txt
