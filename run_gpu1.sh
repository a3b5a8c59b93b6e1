#!/bin/bash
# GPU session: kernel numerics, model parity, HIP bench. Stops on any fault/timeout.
mkdir -p gpurun_out && python -m chiaswarm_amd._build
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_hip.log 2>&1
