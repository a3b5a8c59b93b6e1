#!/bin/bash
# Same-box A/B of two kernel-library builds: chiaswarm_amd/lib/ab/libcsk_old.so (A) vs the
# in-tree libcsk.so (B): conv tile probes and the hipGraph UNet step, interleaved A B A B.
TAG=${1:-x}
mkdir -p gpurun_out
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 > gpurun_out/libab_${TAG}_step_$arm.log 2>&1 || exit 1
  echo "$arm $(grep median gpurun_out/libab_${TAG}_step_$arm.log)"
done
for arm in A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 200 python tools/tilebench.py --tiles 26 --only conv --gn --rounds 2 > gpurun_out/libab_${TAG}_tb_$arm.txt 2>&1 || exit 1
done
paste <(grep -v amdgpu gpurun_out/libab_${TAG}_tb_A.txt | cut -c1-75) <(grep -v amdgpu gpurun_out/libab_${TAG}_tb_B.txt | cut -c30-75) | head -20
