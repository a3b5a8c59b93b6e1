#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or geglu" --timeout 200 --timeout-method thread > gpurun_out/pytest_f.log 2>&1 || { tail -30 gpurun_out/pytest_f.log; exit 1; }
tail -2 gpurun_out/pytest_f.log
timeout -k 10 300 python tools/gemmprof.py --shapes 32768x320x2560:geglu,8192x640x5120:geglu,2048x1280x10240:geglu,32768x320x320,8192x640x640,2048x1280x1280 --tiles 11,12,13,14,17,18,19,20,21,22,23,24 > gpurun_out/gemmprof_f.log 2>&1 || exit $?
timeout -k 10 400 python tools/retune.py --drop '^g:(32768|8192|2048):' --out gpurun_out/tune_f.json > gpurun_out/retune_f.log 2>&1 || exit $?
cp gpurun_out/tune_f.json chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_f.log 2>&1 || exit $?
tail -1 gpurun_out/bench_f.log
