#!/bin/bash
# Short-KV attention: isolated timings per kernel / rows, numerics, step A/B; batch-1 latency with the batch-2 table.
TAG=${1:-x}
mkdir -p gpurun_out
for shape in 8,4096,77,5,64 8,1024,77,10,64 8,256,77,20,64 2,4096,77,5,64; do
  for kv in "2 0" "3 64" "3 128" "3 256"; do
    set -- $kv
    timeout -k 10 60 python tools/attnbench.py --short-kv $1 --kv-rows $2 --iters 50 --shape $shape 2>&1 | grep -v amdgpu.ids >> gpurun_out/r3j_attn_$TAG.txt || exit 1
  done
done
cat gpurun_out/r3j_attn_$TAG.txt
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k "attention" > gpurun_out/r3j_kern_$TAG.log 2>&1 || { tail -40 gpurun_out/r3j_kern_$TAG.log; exit 1; }
tail -1 gpurun_out/r3j_kern_$TAG.log
timeout -k 10 250 python tools/abstep.py --arms xkv2,kvr64,kvr128,kvr256 --rounds 5 > gpurun_out/r3j_ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3j_ab_$TAG.txt; exit 1; }
grep median gpurun_out/r3j_ab_$TAG.txt
timeout -k 10 200 python tools/bench_configs.py --only sd21-b1 --reps 3 > gpurun_out/r3j_b1_$TAG.log 2>&1 || { tail -20 gpurun_out/r3j_b1_$TAG.log; exit 1; }
grep "{" gpurun_out/r3j_b1_$TAG.log | cut -c1-300
