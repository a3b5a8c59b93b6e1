#!/bin/bash
# Split-KV attention threshold (aswN arms) at CFG batch 2 and 8.
mkdir -p gpurun_out
timeout -k 10 300 python tools/abstep.py --batch 2 --arms asw512,asw1024,asw2048,asw0 --rounds 5 > gpurun_out/ab_asw_b2_r5p.log 2>&1 || { tail -20 gpurun_out/ab_asw_b2_r5p.log; exit 1; }
tail -4 gpurun_out/ab_asw_b2_r5p.log
timeout -k 10 300 python tools/abstep.py --arms asw512,asw1024,asw2048 --rounds 5 > gpurun_out/ab_asw_b8_r5p.log 2>&1 || { tail -20 gpurun_out/ab_asw_b8_r5p.log; exit 1; }
tail -3 gpurun_out/ab_asw_b8_r5p.log
