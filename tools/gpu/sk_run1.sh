set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_sk_gpu.py -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sk_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/sk_tests.log | head -30; exit $rc; }
timeout -k 10 400 python tools/tilebench.py --tiles 13,18,20,40,41,42,43 --only gemm --res --rounds 3 > gpurun_out/tb_sk1.txt 2>&1 || { tail -20 gpurun_out/tb_sk1.txt; exit 1; }
cat gpurun_out/tb_sk1.txt
rm -f gpurun_out/fa_ab.log
for p in 0 512 0 512 640; do
  timeout -k 10 60 python tools/attnbench.py --shape 8,4096,4096,5,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
done
timeout -k 10 60 python tools/attnbench.py --shape 8,1024,1024,10,64 --probe 512 --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
cat gpurun_out/fa_ab.log
