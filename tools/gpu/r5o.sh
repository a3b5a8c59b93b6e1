#!/bin/bash
# CFG-batch-2 conv_in (B1) on a 64-row tile: GN fallbacks at batch 2 and 8, and the batch-2 step A/B.
mkdir -p gpurun_out
for b in 2 8; do
  timeout -k 10 200 python tools/gn_fallbacks.py --batch $b > gpurun_out/gn_fallbacks_b${b}_r5o.log 2>&1 || { tail -20 gpurun_out/gn_fallbacks_b${b}_r5o.log; exit 1; }
  echo "batch $b"; grep -v amdgpu.ids gpurun_out/gn_fallbacks_b${b}_r5o.log
done
python - <<'PY'
import json
t = json.load(open("chiaswarm_amd/lib/tune_gfx950.json"))
del t["c:1:64:64:8:320:3:1:0"]
json.dump(t, open("/tmp/tune_old_r5o.json", "w"))
PY
for arm in new old new old; do
  if [ $arm = old ]; then export CSK_TUNE_FILE=/tmp/tune_old_r5o.json; else unset CSK_TUNE_FILE; fi
  timeout -k 10 150 python tools/abstep.py --batch 2 --arms base --rounds 3 > gpurun_out/ab_${arm}_r5o.log 2>&1 || exit 1
  echo "$arm $(grep median gpurun_out/ab_${arm}_r5o.log)"
done
