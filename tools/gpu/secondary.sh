#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_configs.py > gpurun_out/secondary_r1z.jsonl 2> gpurun_out/secondary_r1z.err || { tail -20 gpurun_out/secondary_r1z.err; exit 1; }
cat gpurun_out/secondary_r1z.jsonl
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/bench_torchrun_r1z.log 2>&1 || { tail -20 gpurun_out/bench_torchrun_r1z.log; exit 1; }
tail -1 gpurun_out/bench_torchrun_r1z.log
