set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python tools/tilebench.py --graph --iters 10 --tiles 11,26,31,32,34,12,13 --only gemm --rounds 3 --gemms "2048,10240,1280:geglu;8192,5120,640:geglu;32768,2560,320:geglu;2048,1280,5120;2048,3840,1280;2048,1280,1280" > gpurun_out/tb_big.txt 2>&1 || { tail -20 gpurun_out/tb_big.txt; exit 1; }
cat gpurun_out/tb_big.txt
