set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_fa_gpu.py -p no:cacheprovider > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -2 gpurun_out/fa_tests.log
for p in 0 1 2 4 8 16 5 12; do
  timeout -k 10 60 python tools/attnbench.py --shape 8,4096,4096,5,64 --probe $p --iters 30 2>/dev/null >> gpurun_out/fa_probe.log || exit 1
done
cat gpurun_out/fa_probe.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/attnbench.py --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/attnbench.py --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1 || exit 1
echo PMC done
