#!/bin/bash
# Channel-blocked GN apply: block width x workgroup target combinations.
mkdir -p gpurun_out


timeout -k 10 300 python tools/abstep.py --arms gcm1+gcb512,gcm2+gcb512,gcm2+gcb1024,gcm2+gcb256,gcm1+gcb1024 --rounds 5 > gpurun_out/ab_gcm_r5g.log 2>&1 || { tail -20 gpurun_out/ab_gcm_r5g.log; exit 1; }
tail -5 gpurun_out/ab_gcm_r5g.log
