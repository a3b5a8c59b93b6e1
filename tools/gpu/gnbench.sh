#!/bin/bash
# GroupNorm apply paths on the UNet shapes (tools/gnbench.py), isolated, graph-replayed.
mkdir -p gpurun_out
timeout -k 10 200 python tools/gnbench.py > gpurun_out/gnbench.txt 2>&1 || { tail -20 gpurun_out/gnbench.txt; exit 1; }
grep -v amdgpu gpurun_out/gnbench.txt
