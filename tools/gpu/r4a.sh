#!/bin/bash
# GroupNorm: prologue-merge threshold (entries per sample merged by every apply workgroup) A/B.
mkdir -p gpurun_out
timeout -k 10 400 python tools/abstep.py --arms gn1024,gn1400,gn5200,gn1024 --rounds 5 > gpurun_out/abstep_gnthr_r4a.txt 2>&1 || { tail -20 gpurun_out/abstep_gnthr_r4a.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/abstep_gnthr_r4a.txt
