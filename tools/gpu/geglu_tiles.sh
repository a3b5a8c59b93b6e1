set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python tools/tilebench.py --tiles 11,15,20,27,31,32,34 --only gemm --rounds 3 --iters 20 --gemms "2048,10240,1280:geglu;8192,5120,640:geglu;32768,2560,320:geglu;512,10240,1280:geglu;2048,1280,5120;2048,3840,1280;8192,1920,640" > gpurun_out/tb_geglu.txt 2>&1 || { tail -20 gpurun_out/tb_geglu.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tb_geglu.txt
