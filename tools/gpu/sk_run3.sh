set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_sk_gpu.py -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1; rc=$?
tail -1 gpurun_out/sk_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/sk_tests.log | head -30; exit $rc; }
timeout -k 10 400 python tools/tilebench.py --tiles 14,18,40,41,42,43 --only gemm --rounds 3 --gemms "512,1280,1280;128,1280,1280;2048,640,640;2048,1280,1280;8192,320,320" > gpurun_out/tb_sk3.txt 2>&1 || { tail -20 gpurun_out/tb_sk3.txt; exit 1; }
grep -v amdgpu gpurun_out/tb_sk3.txt
