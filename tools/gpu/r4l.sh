#!/bin/bash
# Upsample (nearest-x2 fused) conv shapes of the VAE decoder and the SD2.1 UNet: tile sweep.
mkdir -p gpurun_out
timeout -k 10 500 python tools/tilebench.py --only conv --tiles 11,20,26,31,32,33 --rounds 2 --iters 4 \
  --convs "4,64,64,512,512u;4,128,128,512,512u;4,256,256,256,256u;8,32,32,640,640u;8,16,16,1280,1280u;8,8,8,1280,1280u" > gpurun_out/tilebench_up2x_r4l.txt 2>&1 || { tail -20 gpurun_out/tilebench_up2x_r4l.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tilebench_up2x_r4l.txt
