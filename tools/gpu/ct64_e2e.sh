set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/bench_configs.py --only esrgan --reps 7 > gpurun_out/ct64_esr.log 2>&1 || { tail -20 gpurun_out/ct64_esr.log; exit 1; }
grep config gpurun_out/ct64_esr.log
CSK_CONV_TILE64=0 timeout -k 10 300 python tools/bench_configs.py --only esrgan --reps 7 > gpurun_out/ct64_esr0.log 2>&1 || { tail -20 gpurun_out/ct64_esr0.log; exit 1; }
grep config gpurun_out/ct64_esr0.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_tile_gpu.py tests/test_models_gpu.py -k "esrgan or rrdb or conv_tile" -p no:cacheprovider > gpurun_out/ct64_t2.log 2>&1; rc=$?
tail -1 gpurun_out/ct64_t2.log; exit $rc
