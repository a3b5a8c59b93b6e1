set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T=chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 500 python tools/steptune.py --batch 2 --fixup --min-gain-us 10 --budget 400 --out gpurun_out/tune_b2fx3.json > gpurun_out/steptune_b2fx3.log 2>&1 || { tail -20 gpurun_out/steptune_b2fx3.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_b2fx3.log | tail -30
cp $T /tmp/tune_old.json
st() {
  timeout -k 10 200 python tools/steptune.py --batch 2 --budget 1 --out /tmp/x.json > gpurun_out/fx5_$1.log 2>&1 || { tail -20 gpurun_out/fx5_$1.log; return 1; }
  echo "$1 $(grep 'start step' gpurun_out/fx5_$1.log)"
}
for i in 1 2; do
cp gpurun_out/tune_b2fx3.json $T; st fx$i || exit 1
cp /tmp/tune_old.json $T; st base$i || exit 1
done
