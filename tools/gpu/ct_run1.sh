set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_tile_gpu.py -p no:cacheprovider > gpurun_out/ct_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ct_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/ct_tests.log | head -30; exit $rc; }
timeout -k 10 300 python tools/bench_configs.py --only esrgan --reps 5 > gpurun_out/esrgan_ct.jsonl 2> gpurun_out/esrgan_ct.err || { tail -20 gpurun_out/esrgan_ct.err; exit 1; }
cat gpurun_out/esrgan_ct.jsonl
CSK_CONV_TILE=0 timeout -k 10 300 python tools/bench_configs.py --only esrgan --reps 5 >> gpurun_out/esrgan_ct.jsonl 2>> gpurun_out/esrgan_ct.err || { tail -20 gpurun_out/esrgan_ct.err; exit 1; }
tail -1 gpurun_out/esrgan_ct.jsonl
