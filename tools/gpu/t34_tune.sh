set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python tools/steptune.py --model sdxl --batch 2 --latent 128 --only-tiles 34,32 --all-tiles --budget 480 --out gpurun_out/tune_sdxl_t34.json > gpurun_out/steptune_sdxl_t34.log 2>&1 || { tail -20 gpurun_out/steptune_sdxl_t34.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_sdxl_t34.log | tail -30
cp gpurun_out/tune_sdxl_t34.json chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 500 python tools/steptune.py --batch 8 --only-tiles 34,32 --all-tiles --budget 400 --out gpurun_out/tune_b8_t34.json > gpurun_out/steptune_b8_t34.log 2>&1 || { tail -20 gpurun_out/steptune_b8_t34.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_b8_t34.log | tail -30
