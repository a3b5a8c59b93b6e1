set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/fa_spike.py 0,256 > gpurun_out/fa_spike.log 2>&1 || { tail -20 gpurun_out/fa_spike.log; exit 1; }
grep probe gpurun_out/fa_spike.log | cut -c1-120
bash tools/gpu/fa_run6.sh || exit 1
bash tools/gpu/callprof.sh r5a > /dev/null || exit 1
head -30 gpurun_out/callprof_r5a.txt; grep -A30 "torch (at::native)" gpurun_out/callprof_r5a.txt
