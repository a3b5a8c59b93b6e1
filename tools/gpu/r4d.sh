#!/bin/bash
# Per-request time-projection table: loop tests, then a same-box bench A/B (table off / on).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_loop_gpu.py tests/test_models_gpu.py -x -q -k "row_bcast or loop or txt2img or graph_requests" --timeout 200 --timeout-method thread > gpurun_out/pytest_temb_r4d.log 2>&1 || { tail -30 gpurun_out/pytest_temb_r4d.log; exit 1; }
tail -1 gpurun_out/pytest_temb_r4d.log
for arm in 0 1 0 1; do
  CSK_TEMB_TABLE=$arm timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_temb${arm}_r4d.log 2>&1 || exit $?
  echo "temb=$arm $(tail -1 gpurun_out/bench_temb${arm}_r4d.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_job_latency_ms"], d["phase_ms_median"])')"
done
