#!/bin/bash
# Kernel trace + PMC passes over the VAE decode and the text encoder (tools/decodeprof.py).
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/dk_$TAG -o dk -- python3 $R/tools/decodeprof.py --iters 3 > $R/gpurun_out/dk_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/dk_$TAG.log; exit 1; }
grep " ms" $R/gpurun_out/dk_$TAG.log
find /tmp/dk_$TAG -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/dk_${TAG}_kernel_stats.csv \;
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_COUNT"
P3="WRITE_SIZE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  D=/tmp/pmcd_${TAG}_$i
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d $D -o p -- python3 $R/tools/decodeprof.py --iters 1 > $R/gpurun_out/pmcd_${TAG}_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -c 3000 $R/gpurun_out/pmcd_${TAG}_$i.log; exit $rc; fi
  python3 $R/tools/pmc_summary.py $(find $D -name '*.db') > $R/gpurun_out/pmcd_${TAG}_$i.txt || exit $?
done
head -20 $R/gpurun_out/pmcd_${TAG}_1.txt
