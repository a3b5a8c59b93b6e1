#!/bin/bash
# Runtime-knob A/Bs of the hipGraph UNet step, one process per knob group so a
# knob set by one arm never leaks into another group (abstep's settings persist
# into later arms of the same run): bash tools/gpu/knobs.sh TAG BATCH
TAG=${1:-x}
B=${2:-8}
mkdir -p gpurun_out
out=gpurun_out/knobs_${TAG}_b${B}.txt
: > $out
for arms in base,side1 base,swodd0,swodd1 base,band0,band1 base,gnd0,gnd1 base,nt0,nt1 base,skr1,skr8 base,lnk0,lnk1 base,a32off,a32on; do
  echo "## $arms" >> $out
  timeout -k 10 200 python tools/abstep.py --batch $B --arms $arms --rounds 3 2>/dev/null | grep median >> $out || exit 1
done
cat $out
