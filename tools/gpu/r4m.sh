#!/bin/bash
# 8x8-level UNet convs (M = 512 rows): split-K 8 vs 16 on the 256-row / 160-wide tiles.
mkdir -p gpurun_out
timeout -k 10 500 python tools/tilebench.py --only conv --tiles 32,33,26,11 --splits 4,8,16 --rounds 3 --iters 6 \
  --convs "8,8,8,1280,1280;8,8,8,2560,1280;8,16,16,1280,1280" > gpurun_out/tilebench_8x8_r4m.txt 2>&1 || { tail -20 gpurun_out/tilebench_8x8_r4m.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tilebench_8x8_r4m.txt
