#!/bin/bash
# Short-KV cross-attention rows per workgroup (kvrN arms; 0 = auto) at CFG batch 8 and 2.
mkdir -p gpurun_out
timeout -k 10 300 python tools/abstep.py --arms kvr0,kvr64,kvr128,kvr256 --rounds 5 > gpurun_out/ab_kvr_b8_r5t.log 2>&1 || { tail -20 gpurun_out/ab_kvr_b8_r5t.log; exit 1; }
tail -4 gpurun_out/ab_kvr_b8_r5t.log
timeout -k 10 300 python tools/abstep.py --batch 2 --arms kvr0,kvr64,kvr128,kvr256 --rounds 5 > gpurun_out/ab_kvr_b2_r5t.log 2>&1 || { tail -20 gpurun_out/ab_kvr_b2_r5t.log; exit 1; }
tail -4 gpurun_out/ab_kvr_b2_r5t.log
