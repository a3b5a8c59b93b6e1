#!/bin/bash
# Round 5: tune the ESRGAN / ControlNet shapes, then the secondary configs (5 reps) and kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python tools/retune.py --models esrgan,controlnet --out gpurun_out/tune_r5.json > gpurun_out/retune_r5.log 2>&1 || { tail -20 gpurun_out/retune_r5.log; exit 1; }
grep -c measured gpurun_out/retune_r5.log
cp gpurun_out/tune_r5.json chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 600 python tools/bench_configs.py --only sdxl,controlnet,esrgan,sd21-b1 --reps 5 > gpurun_out/secondary_r5.jsonl 2> gpurun_out/secondary_r5.err || { tail -20 gpurun_out/secondary_r5.err; exit 1; }
cat gpurun_out/secondary_r5.jsonl
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_esrgan -o es -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --only esrgan --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_esrgan.log 2>&1 || exit 1
echo esrgan-prof-ok
