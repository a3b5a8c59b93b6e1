set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T=chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 780 python tools/steptune.py --model sdxl --batch 2 --latent 128 --min-gain-us 15 --budget 660 --out gpurun_out/tune_sdxl2.json > gpurun_out/steptune_sdxl2.log 2>&1 || { tail -20 gpurun_out/steptune_sdxl2.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_sdxl2.log | tail -30
