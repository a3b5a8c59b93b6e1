#!/bin/bash
# PMC counters of one conv/GEMM tile (tools/convbench.py), one counter pass per run.
# usage: bash tools/gpu/pmc_gemm.sh TAG "convbench args"
TAG=${1:-x}
ARGS=${2:-"--tiles 11 --iters 5"}
mkdir -p gpurun_out
export TMPDIR=/tmp
export CSK_ENCODER_PROCS=0
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $GRAFT_REPO_ROOT/gpurun_out/pmcg_${TAG}_$i -o p -- python3 $GRAFT_REPO_ROOT/tools/convbench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/pmcg_${TAG}_$i.log 2>&1 || exit $?
done
