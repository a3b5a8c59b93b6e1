#!/bin/bash
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 250 python tools/abstep.py --arms gnwg512,gnwg1024,gnwg2048,gnwg256 --rounds 5 > gpurun_out/r3n_ab_$TAG.txt 2>&1 || { tail -20 gpurun_out/r3n_ab_$TAG.txt; exit 1; }
grep median gpurun_out/r3n_ab_$TAG.txt
