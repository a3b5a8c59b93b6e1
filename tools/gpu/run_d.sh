#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or norm or gemm or conv" --timeout 200 --timeout-method thread > gpurun_out/pytest_d.log 2>&1 || { tail -30 gpurun_out/pytest_d.log; exit 1; }
tail -2 gpurun_out/pytest_d.log
timeout -k 10 300 python tools/opbench.py --filter attn --out gpurun_out/opbench_attn_d.json > gpurun_out/opbench_attn_d.log 2>&1 || exit $?
timeout -k 10 300 python tools/opbench.py --filter norm --out gpurun_out/opbench_norm_d.json > gpurun_out/opbench_norm_d.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_d.log 2>&1 || exit $?
tail -1 gpurun_out/bench_d.log
