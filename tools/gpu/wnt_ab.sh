set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/abstep.py --arms wnt0,wnt1 --rounds 5 > gpurun_out/abstep_wnt_b8.log 2>&1 || { tail -20 gpurun_out/abstep_wnt_b8.log; exit 1; }
tail -3 gpurun_out/abstep_wnt_b8.log
timeout -k 10 300 python tools/abstep.py --arms wnt0,wnt1 --rounds 5 --batch 2 > gpurun_out/abstep_wnt_b2.log 2>&1 || { tail -20 gpurun_out/abstep_wnt_b2.log; exit 1; }
tail -3 gpurun_out/abstep_wnt_b2.log
