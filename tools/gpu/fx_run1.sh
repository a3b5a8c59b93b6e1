set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_fixup_gpu.py -p no:cacheprovider > gpurun_out/fx_tests.log 2>&1; rc=$?
tail -3 gpurun_out/fx_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/fx_tests.log | head -30; exit $rc; }
timeout -k 10 400 python tools/tilebench.py --tiles 14,18,12 --splits 1,2,4,8,-2,-4,-8 --only gemm --rounds 3 --gemms "128,1280,1280;512,1280,1280;128,1280,5120;512,1280,5120;2048,640,640;512,3840,1280" > gpurun_out/tb_fx1.txt 2>&1 || { tail -20 gpurun_out/tb_fx1.txt; exit 1; }
cat gpurun_out/tb_fx1.txt
