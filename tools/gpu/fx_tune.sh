set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 660 python tools/steptune.py --batch 2 --fixup --budget 560 --out gpurun_out/tune_b2fx.json > gpurun_out/steptune_b2fx.log 2>&1 || { tail -20 gpurun_out/steptune_b2fx.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_b2fx.log | tail -30
cp gpurun_out/tune_b2fx.json chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 560 python tools/steptune.py --batch 8 --fixup --budget 460 --out gpurun_out/tune_b8fx.json > gpurun_out/steptune_b8fx.log 2>&1 || { tail -20 gpurun_out/steptune_b8fx.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_b8fx.log | tail -30
