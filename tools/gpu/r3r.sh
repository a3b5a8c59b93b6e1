#!/bin/bash
# Attention QT1/QT2 at the half-batch shape; GEMM epilogue cost with a residual input.
mkdir -p gpurun_out
for v in 5 7 6; do
  timeout -k 10 120 python tools/attnbench.py --shape 4,4096,4096,5,64 --variant $v >> gpurun_out/attn_b4_r3r.txt 2>&1 || exit $?
done
for v in 5 7; do
  timeout -k 10 120 python tools/attnbench.py --shape 8,1024,1024,10,64 --variant $v >> gpurun_out/attn_b4_r3r.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/attn_b4_r3r.txt
timeout -k 10 300 python tools/tilebench.py --only gemm --tiles 19,20,13,11 --probe --res --rounds 3 \
  --gemms "32768,320,320;8192,640,640;2048,1280,1280;32768,320,1280" > gpurun_out/tilebench_res_r3r.txt 2>&1 || { tail -5 gpurun_out/tilebench_res_r3r.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tilebench_res_r3r.txt
