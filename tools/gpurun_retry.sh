#!/bin/bash
# Host-side helper: run a gpurun call, re-submitting ONLY when gpurun reports an
# infrastructure transient (nothing ran, nothing charged).  usage: gpurun_retry.sh OUTFILE TIMEOUT CMD
OUT=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6; do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > "$OUT" 2>&1
  if grep -q "status=transient" "$OUT" && ! grep -q "charged=[1-9]" "$OUT"; then
    sleep 45
    continue
  fi
  exit 0
done
