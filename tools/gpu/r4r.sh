#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dup2" --timeout 120 --timeout-method thread > gpurun_out/pytest_dup2_r4r.log 2>&1 || { tail -30 gpurun_out/pytest_dup2_r4r.log; exit 1; }
tail -1 gpurun_out/pytest_dup2_r4r.log
timeout -k 10 120 python - > gpurun_out/dup2_time_r4r.txt 2>&1 <<'P' || exit 1
import torch
from chiaswarm_amd.ops import _lib, hip_ops
_lib.load()
x = torch.randn(4, 64, 64, 320, device="cuda").bfloat16()
for name, fn in (("dup2", lambda: hip_ops.dup2(x)), ("cat", lambda: torch.cat([x, x]))):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): fn()
    e1.record(); torch.cuda.synchronize()
    print(name, round(e0.elapsed_time(e1) / 50 * 1000, 1), "us")
P
cat gpurun_out/dup2_time_r4r.txt | grep -v amdgpu
