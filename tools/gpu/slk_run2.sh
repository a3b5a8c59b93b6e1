set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/tilebench.py --tiles 14,18,42,43,44 --splits 1,2,4 --only gemm --rounds 3 --gemms "128,1280,1280;512,1280,1280;128,1280,5120;512,1280,5120;512,320,1024;128,1280,2560" > gpurun_out/tb_slk2.txt 2>&1 || { tail -20 gpurun_out/tb_slk2.txt; exit 1; }
cat gpurun_out/tb_slk2.txt
