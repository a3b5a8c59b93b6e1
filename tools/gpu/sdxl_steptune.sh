set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 700 python tools/steptune.py --model sdxl --batch 2 --latent 128 --keys "g:2048:" --budget 600 --out gpurun_out/tune_sdxl_step.json > gpurun_out/steptune_sdxl.log 2>&1 || { tail -20 gpurun_out/steptune_sdxl.log; exit 1; }
tail -25 gpurun_out/steptune_sdxl.log
