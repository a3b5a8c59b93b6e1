set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/bench_configs.py --only sd21-b1 --reps 5 > gpurun_out/ab_b1_new.log 2>&1 || { tail -20 gpurun_out/ab_b1_new.log; exit 1; }
grep config gpurun_out/ab_b1_new.log
CSK_LIB_PATH=$PWD/chiaswarm_amd/lib/libcsk_old.so CSK_ALLOW_STALE=1 timeout -k 10 300 python tools/bench_configs.py --only sd21-b1 --reps 5 > gpurun_out/ab_b1_old.log 2>&1 || { tail -20 gpurun_out/ab_b1_old.log; exit 1; }
grep config gpurun_out/ab_b1_old.log
timeout -k 10 300 python tools/bench_configs.py --only sd21-b1 --reps 5 > gpurun_out/ab_b1_new2.log 2>&1 || { tail -20 gpurun_out/ab_b1_new2.log; exit 1; }
grep config gpurun_out/ab_b1_new2.log
