set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for nt in 0 1 2; do
timeout -k 10 300 python tools/tilebench.py --nt $nt --graph --iters 10 --tiles 19,18,11,12 --only gemm --rounds 3 --res --gemms "32768,320,320;32768,960,320;8192,640,640;2048,1280,1280" > gpurun_out/tb_nt$nt.txt 2>&1 || { tail -20 gpurun_out/tb_nt$nt.txt; exit 1; }
echo "== nt$nt"; grep -v amdgpu gpurun_out/tb_nt$nt.txt
done
timeout -k 10 400 python tools/abstep.py --arms nt0,nt1,nt2 --rounds 4 > gpurun_out/abstep_nt.log 2>&1 || { tail -20 gpurun_out/abstep_nt.log; exit 1; }
tail -6 gpurun_out/abstep_nt.log
