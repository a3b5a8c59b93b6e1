set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T=chiaswarm_amd/lib/tune_gfx950.json
cp $T /tmp/tune_new.json
run() {  # $1 tag
  timeout -k 10 300 python tools/bench_configs.py --only sd21-b1 --reps 5 > gpurun_out/ab3_$1.log 2>&1 || { tail -20 gpurun_out/ab3_$1.log; return 1; }
  echo "$1 $(grep config gpurun_out/ab3_$1.log)"
  timeout -k 10 200 python tools/steptune.py --batch 2 --budget 1 --out /tmp/x.json > gpurun_out/ab3_st_$1.log 2>&1 || { tail -20 gpurun_out/ab3_st_$1.log; return 1; }
  echo "$1 $(grep 'start step' gpurun_out/ab3_st_$1.log)"
}
run new1 || exit 1
cp tools/gpu/data/tune_pre_fixup.json $T
CSK_LIB_PATH=$PWD/chiaswarm_amd/lib/libcsk_old.so CSK_ALLOW_STALE=1 run old || exit 1
cp /tmp/tune_new.json $T
run new2 || exit 1
