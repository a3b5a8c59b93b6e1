#!/bin/bash
# Same-box step A/B: the in-tree library vs chiaswarm_amd/lib/ab/libcsk_old.so (interleaved arms).
TAG=${1:-x}
ARMS=${ARMS:-base}
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
OLD=$R/chiaswarm_amd/lib/ab/${OLDLIB:-libcsk_old.so}
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms $ARMS --rounds 3 > gpurun_out/libab_${TAG}_$arm.log 2>&1 || { tail -5 gpurun_out/libab_${TAG}_$arm.log; exit 1; }
  echo "$arm $(grep median gpurun_out/libab_${TAG}_$arm.log)"
done
