#!/bin/bash
# conv_in epilogue GN statistics + dup2 keeps them: model / ControlNet tests, step time, per-call profile.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "unet or vae or control or dup2 or group_norm" > gpurun_out/tests_r5b.log 2>&1 || { tail -30 gpurun_out/tests_r5b.log; exit 1; }
tail -2 gpurun_out/tests_r5b.log
timeout -k 10 200 python tools/abstep.py --arms base --rounds 5 > gpurun_out/ab_r5b.log 2>&1 || { tail -20 gpurun_out/ab_r5b.log; exit 1; }
tail -2 gpurun_out/ab_r5b.log
bash tools/gpu/callprof.sh r5b > /dev/null && grep -E "csk_group_norm|device time" gpurun_out/callprof_r5b.txt
