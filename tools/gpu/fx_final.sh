set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_fixup_gpu.py tests/test_models_gpu.py -p no:cacheprovider > gpurun_out/fxf_tests.log 2>&1; rc=$?
tail -1 gpurun_out/fxf_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/fxf_tests.log | head -30; exit $rc; }
timeout -k 10 400 python tools/bench_configs.py --only sd21-b1,controlnet --reps 5 > gpurun_out/fxf_b1.log 2>&1 || { tail -20 gpurun_out/fxf_b1.log; exit 1; }
grep config gpurun_out/fxf_b1.log
