#!/bin/bash
# Round 4: epilogue operand prefetch (residual / bias rows issued per fragment
# pair before its stores) - same-box A/B of the HEAD library (A) vs the tree (B):
# GEMMs with a residual input, then the SD2.1 step at CFG batch 8 and 2; then the
# mid-size GEMM tile / split sweep.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
G="2048,1280,1280;32768,320,320;8192,640,640;32768,320,1280"
for arm in A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 200 python tools/tilebench.py --only gemm --gemms "$G" --tiles 11,13,19,20,26 --res --rounds 3 > $O/r6k_tb_$arm.txt 2>&1 || { tail $O/r6k_tb_$arm.txt; exit 1; }
  echo "== $arm"; grep -v amdgpu $O/r6k_tb_$arm.txt
done
for b in 8 2; do
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > $O/r6k_step.log 2>&1 || { tail $O/r6k_step.log; exit 1; }
  echo "batch $b $arm $(grep median $O/r6k_step.log)"
done
done
unset CSK_LIB_PATH CSK_ALLOW_STALE
timeout -k 10 400 python tools/tilebench.py --only gemm --gemms "2048,1280,1280;8192,640,640;2048,3840,1280;2048,1280,5120" \
  --tiles 11,12,13,14,17,18,19,20,26,27,28,29,33 --splits 1,2,4 --probe --res --rounds 3 > $O/r6k_tiles_$TAG.txt 2>&1 || { tail -20 $O/r6k_tiles_$TAG.txt; exit 1; }
grep -v amdgpu $O/r6k_tiles_$TAG.txt
