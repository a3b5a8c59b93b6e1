set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_tile_gpu.py -p no:cacheprovider > gpurun_out/ct64_tests.log 2>&1; rc=$?
tail -2 gpurun_out/ct64_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/ct64_tests.log | head -30; exit $rc; }
timeout -k 10 300 python tools/convtilebench.py --shapes "512,64,32;512,160,32;512,192,64;512,64,64;1024,64,64;2048,64,64" > gpurun_out/ct64_bench.txt 2>&1 || { tail -20 gpurun_out/ct64_bench.txt; exit 1; }
grep -v amdgpu gpurun_out/ct64_bench.txt
