set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pst_gpu.py -p no:cacheprovider > gpurun_out/pst_tests.log 2>&1; rc=$?
tail -2 gpurun_out/pst_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pst_tests.log | head -30; exit $rc; }
timeout -k 10 400 python tools/tilebench.py --graph --iters 10 --tiles 19,50,18,51 --only gemm --rounds 3 --res --gemms "32768,320,320;32768,960,320;8192,640,640;2048,1280,1280" > gpurun_out/tb_pst2.txt 2>&1 || { tail -20 gpurun_out/tb_pst2.txt; exit 1; }
grep -v amdgpu gpurun_out/tb_pst2.txt
