set -o pipefail
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/fa_probe.log
for p in 0 64 76 77 2 18; do
  timeout -k 10 60 python tools/attnbench.py --shape 8,4096,4096,5,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_probe.log || exit 1
done
cat gpurun_out/fa_probe.log
