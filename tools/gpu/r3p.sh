#!/bin/bash
# CFG-shared prefix: GPU tests, step A/B (dup0 = unshared, dup1 = shared), in-step tuning of the new half-batch shapes.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -v -k "cfg_shared or sd21_parity or txt2img" --timeout 200 --timeout-method thread > gpurun_out/pytest_r3p.log 2>&1 || { tail -30 gpurun_out/pytest_r3p.log; exit 1; }
grep -E "passed|failed|parity" gpurun_out/pytest_r3p.log | tail -8
timeout -k 10 300 python tools/abstep.py --arms dup0,dup1 --rounds 5 > gpurun_out/abstep_dup_r3p.txt 2>&1 || { tail -20 gpurun_out/abstep_dup_r3p.txt; exit 1; }
cat gpurun_out/abstep_dup_r3p.txt
timeout -k 10 700 python -u tools/steptune.py --missing --budget 560 --out gpurun_out/tune_dup_r3p.json > gpurun_out/steptune_dup_r3p.log 2>&1 || { tail -20 gpurun_out/steptune_dup_r3p.log; exit 1; }
tail -25 gpurun_out/steptune_dup_r3p.log
