#!/bin/bash
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 250 python tools/abstep.py --arms gfw1024,gfw0,gfw256 --rounds 7 > gpurun_out/r3l_ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3l_ab_$TAG.txt; exit 1; }
grep median gpurun_out/r3l_ab_$TAG.txt
