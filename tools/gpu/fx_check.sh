set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/bench_configs.py --only sd21-b1 --reps 5 > gpurun_out/fx_b1.log 2>&1 || { tail -20 gpurun_out/fx_b1.log; exit 1; }
tail -3 gpurun_out/fx_b1.log
timeout -k 10 700 python tools/steptune.py --model sdxl --batch 2 --latent 128 --fixup --budget 560 --out gpurun_out/tune_sdxl_fx.json > gpurun_out/steptune_sdxl_fx.log 2>&1 || { tail -20 gpurun_out/steptune_sdxl_fx.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_sdxl_fx.log | tail -30
