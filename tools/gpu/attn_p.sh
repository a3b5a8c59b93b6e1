#!/bin/bash
# Attention tests + variant timing + UNet step vs the old tree (cmp_old/), same box.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 200 --timeout-method thread > gpurun_out/pytest_p.log 2>&1 || { tail -30 gpurun_out/pytest_p.log; exit 1; }
tail -1 gpurun_out/pytest_p.log
for v in 2 3 4 5; do timeout -k 10 120 python tools/attnbench.py --variant $v --iters 50 || exit $?; done
timeout -k 10 120 python tools/attnbench.py --variant 3 --iters 50 --shape 8,1024,1024,10,64 || exit $?
if [ -d cmp_old ]; then
  timeout -k 10 120 python cmp_old/tools/abstep.py --arms base --rounds 3 > gpurun_out/cmp_old_p.log 2>&1 || exit $?
  grep median gpurun_out/cmp_old_p.log
fi
timeout -k 10 120 python tools/abstep.py --arms base --rounds 3 > gpurun_out/abstep_p.log 2>&1 || exit $?
grep median gpurun_out/abstep_p.log
