#!/bin/bash
# bench.py under torch.distributed.run (RCCL group, N=1) as the driver launches it for N > 1.
mkdir -p gpurun_out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/bench_torchrun_r4x.log 2>&1 || { tail -30 gpurun_out/bench_torchrun_r4x.log; exit 1; }
grep '^{' gpurun_out/bench_torchrun_r4x.log | cut -c1-400
