set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for b in 2 8; do
timeout -k 10 200 python tools/steptune.py --batch $b --budget 1 --out gpurun_out/ab_new.json > gpurun_out/ab_new_$b.log 2>&1 || { tail -20 gpurun_out/ab_new_$b.log; exit 1; }
grep "start step" gpurun_out/ab_new_$b.log
CSK_LIB_PATH=$PWD/chiaswarm_amd/lib/libcsk_old.so CSK_ALLOW_STALE=1 timeout -k 10 200 python tools/steptune.py --batch $b --budget 1 --out gpurun_out/ab_old.json > gpurun_out/ab_old_$b.log 2>&1 || { tail -20 gpurun_out/ab_old_$b.log; exit 1; }
grep "start step" gpurun_out/ab_old_$b.log
done
