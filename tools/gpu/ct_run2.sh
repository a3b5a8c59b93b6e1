set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/convtilebench.py > gpurun_out/ctbench.txt 2>&1 || { tail -20 gpurun_out/ctbench.txt; exit 1; }
grep conv gpurun_out/ctbench.txt
