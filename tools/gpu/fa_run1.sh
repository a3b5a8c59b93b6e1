set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attn_fa_gpu.py -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1
rc=$?
tail -5 gpurun_out/fa_tests.log
if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
for sh in 8,4096,4096,5,64 8,1024,1024,10,64 8,256,256,20,64 2,4096,4096,5,64 2,1024,1024,10,64 2,4096,4096,10,64 2,1024,1024,20,64; do
  timeout -k 10 60 python tools/attnbench.py --shape $sh --fa 1 --iters 30 >> gpurun_out/fa_bench.log 2>&1 || exit 1
  timeout -k 10 60 python tools/attnbench.py --shape $sh --fa 0 --iters 30 >> gpurun_out/fa_bench.log 2>&1 || exit 1
done
cat gpurun_out/fa_bench.log
