#!/bin/bash
# Checkpoint: full GPU suite, smoke, headline bench, secondary configs (usage: bash tools/gpu/checkpoint.sh TAG).
TAG=${1:-x}
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/r6u_suite_$TAG.log 2>&1; rc=$?
tail -3 $O/r6u_suite_$TAG.log
grep -E "FAILED|ERROR" $O/r6u_suite_$TAG.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r6u_smoke_$TAG.log 2>&1 || { tail -20 $O/r6u_smoke_$TAG.log; exit 1; }
tail -1 $O/r6u_smoke_$TAG.log
timeout -k 10 600 python bench.py > $O/r6u_bench_$TAG.json 2> $O/r6u_bench_$TAG.err || { tail -20 $O/r6u_bench_$TAG.err; exit 1; }
cat $O/r6u_bench_$TAG.json
timeout -k 10 600 python tools/bench_configs.py --only sd21-b1,sdxl,controlnet,esrgan --reps 3 > $O/r6u_cfg_$TAG.jsonl 2> $O/r6u_cfg_$TAG.err || { tail -20 $O/r6u_cfg_$TAG.err; exit 1; }
cat $O/r6u_cfg_$TAG.jsonl
