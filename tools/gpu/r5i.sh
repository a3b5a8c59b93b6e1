#!/bin/bash
# Short-KV cross-attention: Q load issued before the K/V staging, K/V loads batched. Tests, then
# same-box A/B of the library builds (A: previous attention.hip) on the UNet step.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > gpurun_out/attn_tests_r5i.log 2>&1 || { tail -30 gpurun_out/attn_tests_r5i.log; exit 1; }
tail -1 gpurun_out/attn_tests_r5i.log
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/libab_r5i_step_$arm.log 2>&1 || exit 1
  echo "$arm $(grep median gpurun_out/libab_r5i_step_$arm.log)"
done
