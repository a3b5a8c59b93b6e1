#!/bin/bash
# End-of-round check: bounds-checking build over the attention-fusion tests, then
# the full GPU suite, smoke, headline bench and secondary configs (release build).
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
CSK_DEBUG=1 timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_qattn.py tests/test_xattn.py > $O/fc_debug_$TAG.log 2>&1 || { tail -30 $O/fc_debug_$TAG.log; exit 1; }
tail -1 $O/fc_debug_$TAG.log
bash tools/gpu/checkpoint.sh $TAG
