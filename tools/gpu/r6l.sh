#!/bin/bash
# Round 4: epilogue operand prefetch + compile-time band store path of the
# LDS-staged epilogue: GEMM/conv numerics, then same-box A/B of the HEAD library
# (A) vs the tree (B: band path on / off arms): tiles 26 / 33 / 19 / 11 with
# residual and GN statistics, then the SD2.1 step at CFG batch 8 and 2.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_xattn.py > $O/r6l_test_$TAG.log 2>&1 || { tail -30 $O/r6l_test_$TAG.log; exit 1; }
tail -2 $O/r6l_test_$TAG.log
G="8192,640,640;32768,320,320;32768,320,1280;2048,1280,1280"
C="8,32,32,640,640;8,64,64,320,320;8,16,16,1280,1280"
for arm in A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 300 python tools/tilebench.py --gemms "$G" --convs "$C" --tiles 11,19,26,33 --res --gn --rounds 3 > $O/r6l_tb_$arm.txt 2>&1 || { tail $O/r6l_tb_$arm.txt; exit 1; }
  echo "== $arm"; grep -v amdgpu $O/r6l_tb_$arm.txt
done
unset CSK_LIB_PATH CSK_ALLOW_STALE
timeout -k 10 200 python tools/abstep.py --arms band0,band1 --rounds 3 > $O/r6l_band.log 2>&1 || { tail $O/r6l_band.log; exit 1; }
grep median $O/r6l_band.log
for b in 8 2; do
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > $O/r6l_step.log 2>&1 || { tail $O/r6l_step.log; exit 1; }
  echo "batch $b $arm $(grep median $O/r6l_step.log)"
done
done
