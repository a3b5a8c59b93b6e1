#!/bin/bash
# Round 4: LDS-staged epilogue issues the next residual vector before the current
# store (the 128x160 / 256-row tiles' generic loop): tree library (A) vs
# lib/ab/libcsk_new.so (B) — GEMM/conv numerics of B, residual GEMMs on tiles
# 26 / 33, then the SD2.1 step at CFG batch 8 and 2, interleaved.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
NEW=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_new.so
CSK_LIB_PATH=$NEW CSK_ALLOW_STALE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "tile or gemm or conv" > $O/r6p_test_$TAG.log 2>&1 || { tail -30 $O/r6p_test_$TAG.log; exit 1; }
tail -1 $O/r6p_test_$TAG.log
G="8192,640,640;32768,320,1280;32768,320,320"
for arm in A B; do
  if [ $arm = B ]; then export CSK_LIB_PATH=$NEW CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 200 python tools/tilebench.py --only gemm --gemms "$G" --tiles 26,33 --res --rounds 3 > $O/r6p_tb_$arm.txt 2>&1 || { tail $O/r6p_tb_$arm.txt; exit 1; }
  echo "== $arm"; grep -v amdgpu $O/r6p_tb_$arm.txt
done
for b in 8 2; do
for arm in A B A B; do
  if [ $arm = B ]; then export CSK_LIB_PATH=$NEW CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > $O/r6p_step.log 2>&1 || { tail $O/r6p_step.log; exit 1; }
  echo "batch $b $arm $(grep median $O/r6p_step.log)"
done
done
