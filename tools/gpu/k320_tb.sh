set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 500 python tools/tilebench.py --graph --iters 10 --tiles 11,12,13,14,18,19,20,26,29,34,36 --only gemm --rounds 3 --res --probe --gemms "32768,320,320;32768,960,320;32768,320,1280;8192,640,640" > gpurun_out/tb_k320.txt 2>&1 || { tail -20 gpurun_out/tb_k320.txt; exit 1; }
cat gpurun_out/tb_k320.txt
