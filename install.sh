#!/usr/bin/env bash
# Linux installer for an MI355X (gfx950) worker node (reference: install.sh,
# CUDA + pip; here ROCm).  Creates ./venv with --system-site-packages so the
# ROCm PyTorch that ships with the ROCm image / rocm/pytorch container is reused,
# installs the small pure-python dependency set, builds the HIP kernel library
# for gfx950 and runs the CPU test-suite.
set -euo pipefail
cd "$(dirname "$0")"

if ! command -v hipcc >/dev/null 2>&1; then
  echo "hipcc not found: install ROCm (>= 6.4, gfx950 support) first" >&2
  exit 1
fi
PY=${PYTHON:-python3}
"$PY" - <<'PYEOF'
import sys
assert sys.version_info >= (3, 9), "python >= 3.9 required"
import torch
assert torch.version.hip, "a ROCm build of PyTorch is required (torch.version.hip is None)"
print("torch", torch.__version__, "hip", torch.version.hip)
PYEOF

if [ ! -d venv ]; then
  "$PY" -m venv --system-site-packages venv
fi
# shellcheck disable=SC1091
source venv/bin/activate
pip install -r requirements.txt
PYTORCH_ROCM_ARCH=gfx950 python -m chiaswarm_amd._build
python -m pytest tests -q -m "not gpu"
echo
echo "installed. configure with:  python -m swarm.initialize"
echo "run the worker with:        python -m swarm.worker"
