set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/fa_spike.py 0,512 > gpurun_out/fa_spike.log 2>&1 || { tail -20 gpurun_out/fa_spike.log; exit 1; }
grep probe gpurun_out/fa_spike.log | cut -c1-100
rm -f gpurun_out/fa_ab.log
for p in 0 512 0 512; do
  timeout -k 10 60 python tools/attnbench.py --shape 8,4096,4096,5,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
done
timeout -k 10 60 python tools/attnbench.py --shape 8,1024,1024,10,64 --probe 0 --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
timeout -k 10 60 python tools/attnbench.py --shape 8,1024,1024,10,64 --probe 512 --iters 30 2>/dev/null >> gpurun_out/fa_ab.log || exit 1
cat gpurun_out/fa_ab.log
