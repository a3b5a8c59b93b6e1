#!/bin/bash
# Round 4: 64x160 tiles (35 / 36) + epilogue prefetch restricted to the tiles with
# register headroom: numerics, isolated tile comparison on the mid-size GEMMs,
# same-box step A/B against the HEAD library, in-step tuning of tiles 35 / 36.
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
OLD=$GRAFT_REPO_ROOT/chiaswarm_amd/lib/ab/libcsk_old.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_xattn.py > $O/r6m_test_$TAG.log 2>&1 || { tail -30 $O/r6m_test_$TAG.log; exit 1; }
tail -2 $O/r6m_test_$TAG.log
timeout -k 10 300 python tools/tilebench.py --only gemm --gemms "2048,1280,1280;8192,640,640;2048,3840,1280;2048,1280,5120;8192,640,2560;8192,1920,640" \
  --tiles 13,18,19,20,26,35,36 --splits 1 --res --rounds 3 > $O/r6m_tiles_$TAG.txt 2>&1 || { tail -20 $O/r6m_tiles_$TAG.txt; exit 1; }
grep -v amdgpu $O/r6m_tiles_$TAG.txt
for b in 8 2; do
for arm in A B A B; do
  if [ $arm = A ]; then export CSK_LIB_PATH=$OLD CSK_ALLOW_STALE=1; else unset CSK_LIB_PATH CSK_ALLOW_STALE; fi
  timeout -k 10 150 python tools/abstep.py --arms base --rounds 3 --batch $b > $O/r6m_step.log 2>&1 || { tail $O/r6m_step.log; exit 1; }
  echo "batch $b $arm $(grep median $O/r6m_step.log)"
done
done
unset CSK_LIB_PATH CSK_ALLOW_STALE
timeout -k 10 500 python tools/steptune.py --keys g: --only-tiles 35,36 --budget 400 --out $O/tune_step_t35_b8_$TAG.json > $O/r6m_st8_$TAG.log 2>&1 || { tail -20 $O/r6m_st8_$TAG.log; exit 1; }
grep -E "\->|done|start" $O/r6m_st8_$TAG.log
