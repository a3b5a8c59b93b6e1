#!/bin/bash
# VAE decoder 3x3 conv shapes (4 x 512^2 images): tile sweep.
mkdir -p gpurun_out
timeout -k 10 500 python tools/tilebench.py --only conv --tiles 11,20,26,31,32,33,15,27 --rounds 2 --iters 4 \
  --convs "4,512,512,128,128;4,512,512,256,128;4,256,256,256,256;4,256,256,512,256;4,128,128,512,512;4,64,64,512,512" > gpurun_out/tilebench_vae_r4j.txt 2>&1 || { tail -20 gpurun_out/tilebench_vae_r4j.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tilebench_vae_r4j.txt
