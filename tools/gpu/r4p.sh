#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_r4p.log 2>&1 || { tail -20 gpurun_out/bench_r4p.log; exit 1; }
grep '^{' gpurun_out/bench_r4p.log
timeout -k 10 300 python tools/abstep.py --arms base --rounds 5 > gpurun_out/abstep_base_r4p.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/abstep_base_r4p.txt
