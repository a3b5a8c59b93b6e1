set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/fa_spike.py 0 > gpurun_out/fa_spike.log 2>&1 || { tail -20 gpurun_out/fa_spike.log; exit 1; }
grep probe gpurun_out/fa_spike.log | cut -c1-100
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_fa_gpu.py -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -1 gpurun_out/fa_tests.log
rm -f gpurun_out/fa_ab.log
for p in 0 0; do
  timeout -k 10 60 python tools/attnbench.py --shape 8,4096,4096,5,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
done
for p in 0; do
  timeout -k 10 60 python tools/attnbench.py --shape 8,1024,1024,10,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
  timeout -k 10 60 python tools/attnbench.py --shape 2,4096,4096,5,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
  timeout -k 10 60 python tools/attnbench.py --shape 2,4096,4096,10,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
done
cat gpurun_out/fa_ab.log
