#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 python tools/qattnbench.py > gpurun_out/qattnbench.txt 2>&1 || { tail -20 gpurun_out/qattnbench.txt; exit 1; }
grep -v amdgpu gpurun_out/qattnbench.txt
