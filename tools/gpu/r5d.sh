#!/bin/bash
# conv_in (CFG-shared, B4) on a 128-row tile: its GN segments match the skip-concat partner's.
mkdir -p gpurun_out
timeout -k 10 200 python tools/gn_fallbacks.py > gpurun_out/gn_fallbacks_r5d.log 2>&1 || { tail -20 gpurun_out/gn_fallbacks_r5d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gn_fallbacks_r5d.log
python - <<'PY'
import json
t = json.load(open("chiaswarm_amd/lib/tune_gfx950.json"))
t["c:4:64:64:8:320:3:1:0"] = [20, 1, 11368.7]
json.dump(t, open("/tmp/tune_old_r5d.json", "w"))
PY
for arm in new old new old; do
  if [ $arm = old ]; then export CSK_TUNE_FILE=/tmp/tune_old_r5d.json; else unset CSK_TUNE_FILE; fi
  timeout -k 10 200 python tools/abstep.py --arms base --rounds 3 > gpurun_out/ab_${arm}_r5d.log 2>&1 || { tail -20 gpurun_out/ab_${arm}_r5d.log; exit 1; }
  echo "$arm $(tail -1 gpurun_out/ab_${arm}_r5d.log)"
done
