set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T=chiaswarm_amd/lib/tune_gfx950.json
cp tools/gpu/data/tune_sdxl2_candidate.json /tmp/new.json
st() {
  timeout -k 10 200 python tools/steptune.py --batch 8 --budget 1 --out /tmp/x.json > gpurun_out/ab_sdxl2_$1.log 2>&1 || { tail -20 gpurun_out/ab_sdxl2_$1.log; return 1; }
  echo "$1 $(grep 'start step' gpurun_out/ab_sdxl2_$1.log)"
}
for i in 1 2; do
cp /tmp/new.json $T; st new$i || exit 1
cp tools/gpu/data/tune_pre_sdxl2.json $T; st old$i || exit 1
done
