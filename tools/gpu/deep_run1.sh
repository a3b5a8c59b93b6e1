set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T=chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_fixup_gpu.py -p no:cacheprovider > gpurun_out/deep_tests.log 2>&1; rc=$?
tail -2 gpurun_out/deep_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/deep_tests.log | head -30; exit $rc; }
timeout -k 10 500 python tools/steptune.py --batch 2 --only-tiles 45,46,47,48 --min-gain-us 10 --budget 420 --out gpurun_out/tune_b2deep.json > gpurun_out/steptune_b2deep.log 2>&1 || { tail -20 gpurun_out/steptune_b2deep.log; exit 1; }
grep -E "\->|done|start" gpurun_out/steptune_b2deep.log | tail -30
cp $T /tmp/tune_old.json
st() {
  timeout -k 10 200 python tools/steptune.py --batch 2 --budget 1 --out /tmp/x.json > gpurun_out/deep_$1.log 2>&1 || { tail -20 gpurun_out/deep_$1.log; return 1; }
  echo "$1 $(grep 'start step' gpurun_out/deep_$1.log)"
}
for i in 1 2; do
cp gpurun_out/tune_b2deep.json $T; st deep$i || exit 1
cp /tmp/tune_old.json $T; st base$i || exit 1
done
