set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/tilebench.py --tiles 11,15,27 --only gemm --probe --rounds 3 --iters 20 --gemms "2048,10240,1280:geglu;8192,5120,640:geglu;32768,2560,320:geglu;2048,1280,5120;2048,3840,1280" > gpurun_out/tb_geglu_probe.txt 2>&1 || { tail -20 gpurun_out/tb_geglu_probe.txt; exit 1; }
grep -v amdgpu gpurun_out/tb_geglu_probe.txt
