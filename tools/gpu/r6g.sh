#!/bin/bash
# Round 4: fused cross-attention block phase probes vs the unfused chain.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 120 python tools/xattnbench.py --batch 8 > gpurun_out/r6g_xattn_$TAG.txt 2>&1 || { tail -20 gpurun_out/r6g_xattn_$TAG.txt; exit 1; }
grep -v amdgpu gpurun_out/r6g_xattn_$TAG.txt
timeout -k 10 120 python tools/xattnbench.py --batch 2 > gpurun_out/r6g_xattn_b2_$TAG.txt 2>&1 || { tail -20 gpurun_out/r6g_xattn_b2_$TAG.txt; exit 1; }
grep -v amdgpu gpurun_out/r6g_xattn_b2_$TAG.txt
