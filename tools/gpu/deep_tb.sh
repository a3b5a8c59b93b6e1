set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/tilebench.py --graph --iters 20 --tiles 14,18,45,46,47,28 --splits 1,-2,-4 --only gemm --rounds 3 --probe --gemms "2,1280,1280;128,1280,1280;512,1280,1280;2048,640,640;512,1280,5120;2048,640,2560" > gpurun_out/tb_deep.txt 2>&1 || { tail -20 gpurun_out/tb_deep.txt; exit 1; }
cat gpurun_out/tb_deep.txt
