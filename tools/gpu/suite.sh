#!/bin/bash
# GPU suite + smoke + headline bench on a gpurun box (no profiler pass).
# usage: gpurun --timeout 1200 -- bash tools/gpu/suite.sh TAG [pytest selection]
TAG=${1:-x}
SEL=${2:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
