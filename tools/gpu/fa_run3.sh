set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_fa_gpu.py -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -2 gpurun_out/fa_tests.log
rm -f gpurun_out/fa_probe.log
for p in 0 1 4 8 12 16; do
  timeout -k 10 60 python tools/attnbench.py --shape 8,4096,4096,5,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_probe.log || exit 1
done
for sh in 8,1024,1024,10,64 2,4096,4096,5,64 2,4096,4096,10,64 2,1024,1024,20,64; do
  timeout -k 10 60 python tools/attnbench.py --shape $sh --iters 30 2>/dev/null >> gpurun_out/fa_probe.log || exit 1
done
cat gpurun_out/fa_probe.log
