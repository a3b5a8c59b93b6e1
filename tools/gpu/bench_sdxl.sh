set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --config sdxl --steps 3 --warmup 1 > gpurun_out/bench_sdxl_r5.log 2>&1 || { tail -20 gpurun_out/bench_sdxl_r5.log; exit 1; }
tail -1 gpurun_out/bench_sdxl_r5.log
