set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_fixup_gpu.py -p no:cacheprovider > gpurun_out/fx_tests.log 2>&1; rc=$?
tail -1 gpurun_out/fx_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/fx_tests.log | head -30; exit $rc; }
st() {
  timeout -k 10 200 python tools/steptune.py --batch $2 --budget 1 --out /tmp/x.json > gpurun_out/ab5_$1.log 2>&1 || { tail -20 gpurun_out/ab5_$1.log; return 1; }
  echo "$1 $(grep 'start step' gpurun_out/ab5_$1.log)"
}
for b in 2 8; do
st new_b$b $b || exit 1
CSK_LIB_PATH=$PWD/chiaswarm_amd/lib/libcsk_old.so CSK_ALLOW_STALE=1 st old_b$b $b || exit 1
st new2_b$b $b || exit 1
done
