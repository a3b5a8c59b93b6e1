#!/bin/bash
# Channel-blocked GN apply workgroup target (gcbN) with 2-unit blocks, CFG batch 8 and 2.
mkdir -p gpurun_out
timeout -k 10 300 python tools/abstep.py --arms gcb512,gcb384,gcb768,gcb1024 --rounds 5 > gpurun_out/ab_gcb_b8_r5u.log 2>&1 || { tail -20 gpurun_out/ab_gcb_b8_r5u.log; exit 1; }
tail -4 gpurun_out/ab_gcb_b8_r5u.log
timeout -k 10 300 python tools/abstep.py --batch 2 --arms gcb512,gcb384,gcb768,gcb1024 --rounds 5 > gpurun_out/ab_gcb_b2_r5u.log 2>&1 || { tail -20 gpurun_out/ab_gcb_b2_r5u.log; exit 1; }
tail -4 gpurun_out/ab_gcb_b2_r5u.log
