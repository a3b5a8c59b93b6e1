set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_gemm_sk_gpu.py -k "geglu or gemm or model or unet" -p no:cacheprovider > gpurun_out/geglu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/geglu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/geglu_tests.log | head -30; exit $rc; }
bash tools/gpu/geglu_probe.sh
