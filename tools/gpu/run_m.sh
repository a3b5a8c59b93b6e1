#!/bin/bash
mkdir -p gpurun_out
true

timeout -k 10 400 python tools/abstep.py --arms gntile,gnfine,lnoff --rounds 5 > gpurun_out/abstep_m.log 2>&1 || exit $?
cat gpurun_out/abstep_m.log | grep median
