set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T=chiaswarm_amd/lib/tune_gfx950.json
cp tools/gpu/data/tune_pre_fixup.json $T
st() {  # $1 tag
  timeout -k 10 200 python tools/steptune.py --batch 2 --budget 1 --out /tmp/x.json > gpurun_out/ab4_st_$1.log 2>&1 || { tail -20 gpurun_out/ab4_st_$1.log; return 1; }
  echo "$1 $(grep 'start step' gpurun_out/ab4_st_$1.log)"
}
st newlib_oldtab1 || exit 1
CSK_LIB_PATH=$PWD/chiaswarm_amd/lib/libcsk_old.so CSK_ALLOW_STALE=1 st oldlib_oldtab1 || exit 1
st newlib_oldtab2 || exit 1
CSK_LIB_PATH=$PWD/chiaswarm_amd/lib/libcsk_old.so CSK_ALLOW_STALE=1 st oldlib_oldtab2 || exit 1
