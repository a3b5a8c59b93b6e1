set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/fa_spike.py 0,256 2>&1 | tee gpurun_out/fa_spike.log
bash tools/gpu/fa_run6.sh
