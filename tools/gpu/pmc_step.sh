#!/bin/bash
# PMC counters over the whole SD2.1 UNet step (tools/abstep.py, hipGraph replay), one counter pass per run.
# usage: bash tools/gpu/pmc_step.sh TAG
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
export CSK_ENCODER_PROCS=0
cd /tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_COUNT"
P3="WRITE_SIZE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  D=/tmp/pmcs_${TAG}_$i
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d $D -o p -- python3 $GRAFT_REPO_ROOT/tools/abstep.py --arms base --rounds 1 --iters 2 > $GRAFT_REPO_ROOT/gpurun_out/pmcs_${TAG}_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -c 3000 $GRAFT_REPO_ROOT/gpurun_out/pmcs_${TAG}_$i.log; exit $rc; fi
  # the rocpd databases are too big to bring back: keep the per-kernel summary only
  python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $(find $D -name '*.db') > $GRAFT_REPO_ROOT/gpurun_out/pmcs_${TAG}_$i.txt || exit $?
done
