#!/bin/bash
# PMC counters of the attention-only loop (one counter pass per run, kernel trace only).
mkdir -p gpurun_out
export TMPDIR=/tmp
export CSK_ENCODER_PROCS=0
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o p -- python3 $GRAFT_REPO_ROOT/tools/attnbench.py --variant 3 --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_LDS -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o p -- python3 $GRAFT_REPO_ROOT/tools/attnbench.py --variant 3 --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1 || exit $?
