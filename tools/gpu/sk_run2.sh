set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu/fa_ab512.sh || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_sk_gpu.py -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sk_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/sk_tests.log | head -30; exit $rc; }
timeout -k 10 400 python tools/tilebench.py --tiles 13,18,20,42,43 --only gemm --rounds 3 --gemms "32768,320,320;8192,640,640;2048,1280,1280;512,1280,1280;2048,1280,640" > gpurun_out/tb_sk2.txt 2>&1 || { tail -20 gpurun_out/tb_sk2.txt; exit 1; }
cat gpurun_out/tb_sk2.txt
