#!/bin/bash
# Secondary configs on the current tree.
mkdir -p gpurun_out
timeout -k 10 700 python tools/bench_configs.py --only sdxl,controlnet,esrgan,sd21-b1 > gpurun_out/secondary_r5h.log 2>&1 || { tail -20 gpurun_out/secondary_r5h.log; exit 1; }
grep '{' gpurun_out/secondary_r5h.log
