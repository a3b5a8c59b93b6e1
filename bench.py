#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): images/sec for the whole node, SD2.1
512x512, 50-step txt2img, batch 4 per GPU (bf16), plus p50 job latency.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N`` without torchrun env vars spawns N rank processes itself (the
parent never touches the GPU; ranks rendezvous on 127.0.0.1, RCCL on GPUs,
gloo with ``--device cpu``), so ``python bench.py --gpus 8`` and the torchrun
form above measure the same N-rank run; each rank asserts WORLD_SIZE == --gpus.

One "step" = one complete txt2img job per GPU: prompt encoding (OpenCLIP-H,
CFG batch), 50 DPM-Solver++(2M) Karras denoising steps of the full SD2.1 UNet
(865.9M params) on the CFG batch of 8 latents 64x64, VAE decode 512x512, uint8
D2H, and JPEG/base64/sha256 result-envelope encoding (in encoder processes,
overlapped with the next job, joined before the clock stops).  Data-parallel over GPUs
(one process per GPU, weak scaling: 4 images per GPU per step; each rank's
job is an independent request, exactly the reference's one-job-per-GPU node
model, so no collective runs inside the timed region).

Model load (outside the timed region, reported as ``model_load_s``): the
random-init weights are written ONCE as a diffusers-layout safetensors
directory (rank 0, /dev/shm), then every rank loads them through the
production loader: with N > 1 ranks each reads only 1/N of the checkpoint
bytes and one RCCL ``all_gather`` per dtype over xGMI assembles the rest
(parallel/sharded.py); ``load_bytes_read_per_rank`` reports the share read.

``--impl reference`` runs the same models with plain PyTorch ops (hipBLASLt
GEMMs, MIOpen channels-last convs, SDPA) = the diffusers-style eager baseline
("reference-on-MI355X") for the A/B.
"""
from __future__ import annotations

import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import json
import os
import statistics
import sys
import time

import torch

METRIC = ("images/sec (whole node) SD2.1 512×512 50-step txt2img at 1/2/4/8 MI355X; "
          "p50 job latency")
# BASELINE.json configs this script drives: (family, resolution, denoise steps, images per GPU, metric, model label)
CONFIGS = {
    "sd21": ("sd21", 512, 50, 4, METRIC,
             "SD2.1 (stable-diffusion-2-1-base arch: UNet 865.9M + OpenCLIP-H 340.4M + VAE 83.7M)"),
    # config #3: SDXL-base 1024², 30 steps, DP batch 8 across 8 GPUs = one image per rank
    "sdxl": ("sdxl", 1024, 30, 1, "images/sec (whole node) SDXL-base 1024×1024 30-step txt2img, DP batch 1 per "
             "MI355X (BASELINE config #3: DP batch 8 across 8); p50 job latency",
             "SDXL-base 1.0 (stable-diffusion-xl-base-1.0 arch: UNet 2567M + CLIP-L + OpenCLIP-bigG + VAE)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="sd21", choices=sorted(CONFIGS),
                    help="BASELINE config: sd21 (headline, config #2) or sdxl (config #3); "
                         "--batch / --res / --denoise-steps / --family override its values")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU per job")
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--denoise-steps", type=int, default=None)
    ap.add_argument("--family", default=None)
    ap.add_argument("--impl", default="hip", choices=["hip", "reference"])
    ap.add_argument("--guidance", type=float, default=7.5)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--device", default=None)
    ap.add_argument("--through-supervisor", action="store_true",
                    help="drive the real serving path: a fake hive -> Supervisor -> per-GPU ProcessExecutor "
                         "children -> router -> pipeline -> encoder -> result POST")
    a = ap.parse_args()
    fam, res, steps, batch, _, _ = CONFIGS[a.config]
    a.family = a.family or fam
    a.res = a.res or res
    a.denoise_steps = a.denoise_steps or steps
    a.batch = a.batch or batch
    return a


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """``--gpus N`` > 1 without a torchrun environment: start N rank processes
    of this script (before this process touches the GPU), forward rank 0's
    JSON line and return the worst exit code.  Every child is polled: as soon
    as ANY rank exits non-zero the others are terminated (a survivor blocked in
    a collective would otherwise wait out the process-group timeout), and the
    failing rank is named on stderr."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [(r, p.returncode) for r, p in enumerate(procs) if p.returncode not in (None, 0)]
            if bad:
                r, code = bad[0]
                print(f"bench: rank {r} exited with {code}; terminating the other ranks", file=sys.stderr, flush=True)
                for q in procs:
                    if q.poll() is None:
                        q.terminate()
                deadline = time.monotonic() + 20
                while time.monotonic() < deadline and any(q.poll() is None for q in procs):
                    time.sleep(0.1)
                break
            time.sleep(0.2)
        rc = max(abs(p.returncode) if p.returncode is not None else 1 for p in procs)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc


def supervisor_bench(args) -> int:
    """``--through-supervisor``: the config's jobs through the production
    serving path (reference loop: swarm/worker.py:113-163) — an in-process fake
    hive serves them over HTTP, the Supervisor polls it, one ProcessExecutor
    child per GPU runs router -> pipeline -> JPEG envelope, results are POSTed
    back.  This process never touches the GPU.  ``value`` = images/s from the
    first timed poll to the last result POST; p50 = the jobs' own start ->
    envelope time (pipeline_config timings), as in the direct bench."""
    import asyncio
    import tempfile

    root = tempfile.mkdtemp(prefix="csk_supbench_")
    os.environ.setdefault("SDAAS_ROOT", root)
    os.environ["SDAAS_TIMINGS"] = "1"
    from chiaswarm_amd.hive.fake import FakeHive
    from chiaswarm_amd.runtime.worker import ProcessExecutor, Supervisor, group_envs
    from chiaswarm_amd.settings import Settings

    fam, res, steps, batch = args.family, args.res, args.denoise_steps, args.batch
    model = {"sd21": "stabilityai/stable-diffusion-2-1-base", "sdxl": "stabilityai/stable-diffusion-xl-base-1.0",
             "tiny": "tiny/sd"}.get(fam, fam)
    prompts = ["a photograph of an astronaut riding a horse", "a watercolor fox in a snowy forest",
               "a cyberpunk city street at night, neon", "a bowl of ramen, studio lighting"]

    def jobs(n, tag):
        return [{"id": f"{tag}{i}", "model_name": model, "prompt": prompts[i % 4],
                 "negative_prompt": "blurry, low quality", "num_inference_steps": steps, "guidance_scale": args.guidance,
                 "num_images_per_prompt": batch, "height": res, "width": res, "seed": 1000 + i,
                 "content_type": "image/jpeg", "parameters": {"scheduler_type": "DPMSolverMultistepScheduler"}}
                for i in range(n)]

    hive = FakeHive().start()
    st = Settings()
    st.sdaas_uri, st.sdaas_token = hive.base, "bench"
    st.preload = model
    st.max_batch = 1
    n = args.gpus
    devs = ["cpu"] * n if args.device == "cpu" else list(range(n))
    exs = [ProcessExecutor(g, env=e) for g, e in zip(devs, group_envs(n, st))]
    try:
        sup = Supervisor(st, executors=exs)

        async def phase(js):
            hive.jobs = list(js)
            before = len(hive.results)
            t0 = time.monotonic()
            await sup.run(max_polls=1)
            return t0, hive.results[before:], hive.result_times[before:]

        async def both():
            await phase(jobs(max(args.warmup, 1) * n, "w"))  # model load, graph capture
            return await phase(jobs(args.steps * n, "t"))

        t0, results, times = asyncio.run(both())
    finally:
        for e in exs:
            e.close()
        hive.stop()
    bad = [r for r in results if not r.get("artifacts") or "error" in (r.get("pipeline_config") or {})]
    if bad or len(results) != args.steps * n:
        print(f"bench: {len(bad)} failed / {len(results)} results: "
              f"{(bad[0].get('pipeline_config') if bad else None)}", file=sys.stderr)
        return 1
    elapsed = max(times) - t0
    lat = [r["pipeline_config"]["timings"]["total"] for r in results if "timings" in r["pipeline_config"]]
    ips = batch * len(results) / elapsed
    rec = {
        "metric": CONFIGS[args.config][4], "value": round(ips, 4), "unit": "images/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32" if args.device == "cpu" else "bf16",
        "data": "synthetic prompts, random-init weights (no checkpoints offline)",
        "config": {"model": (CONFIGS[args.config][5] if fam == CONFIGS[args.config][0]
                             else f"{fam} (not the {args.config} config)"),
                   "bench_config": args.config, "global_batch": batch * n,
                   "seq_len": (res // 8) ** 2, "parallelism": f"dp{n}", "resolution": f"{res}x{res}",
                   "denoise_steps": steps, "guidance_scale": args.guidance},
        "path": "fake hive HTTP -> Supervisor -> ProcessExecutor child -> router -> StableDiffusion -> "
                "JPEG envelope -> POST /api/results",
        "p50_job_latency_ms": round(1000 * statistics.median(lat), 1) if lat else None,
        "p50_job_latency_note": "child job start -> result envelope (pipeline_config timings.total)",
        "phase_ms_median": {k: round(1000 * statistics.median([r["pipeline_config"]["timings"][k] for r in results
                                                                if k in r["pipeline_config"].get("timings", {})]), 2)
                            for k in (results[0]["pipeline_config"].get("timings") or {})},
        "result_interarrival_ms_p50": round(1000 * statistics.median(
            [b - a for a, b in zip(sorted(times), sorted(times)[1:])]), 1) if len(times) > 1 else None,
    }
    print(json.dumps(rec), flush=True)
    return 0


def main():
    args = parse()
    if args.through_supervisor:
        return supervisor_bench(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    # result encoders are separate processes, started before this process touches the GPU
    from chiaswarm_amd.output.encoder import EncoderPool

    pool = EncoderPool()
    from chiaswarm_amd import ops
    from chiaswarm_amd.parallel import comm
    from chiaswarm_amd.pipelines.sd import StableDiffusion
    from chiaswarm_amd.schedulers import get_scheduler

    rank, local_rank, world = comm.init_distributed(backend="gloo" if args.device == "cpu" else None)
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU required")
    on_gpu = torch.cuda.is_available() and args.device != "cpu"
    device = torch.device("cuda", local_rank) if on_gpu else torch.device("cpu")
    if on_gpu:
        torch.cuda.set_device(device)
        torch.backends.cudnn.benchmark = True
    ops.set_mode(args.impl)
    if args.impl == "hip" and on_gpu:
        ops._lib.load()  # fail loudly: the HIP path must be the one measured

    pipe = StableDiffusion(args.family, device=device, seed=1234)
    if args.no_graphs:
        pipe.use_graphs = False
    load_s, load_bytes, load_read_s, load_gather_s = load_through_checkpoint(pipe, rank, world)

    prompts = ["a photograph of an astronaut riding a horse", "a watercolor fox in a snowy forest",
               "a cyberpunk city street at night, neon", "a bowl of ramen, studio lighting"]

    def job(i):
        g = torch.Generator(device=device).manual_seed(1000 * rank + i)
        sched = get_scheduler("DPMSolverMultistepScheduler", **pipe.family.scheduler_kwargs())
        out = pipe(prompt=prompts[i % len(prompts)], negative_prompt="blurry, low quality",
                   num_inference_steps=args.denoise_steps, guidance_scale=args.guidance,
                   num_images_per_prompt=args.batch, height=args.res, width=args.res,
                   generator=g, scheduler=sched, output_type="uint8")
        # JPEG/base64/sha256 envelope encoding in the encoder processes, overlapped
        # with the next job (joined before the clock stops)
        return pool.submit(list(out.images.numpy()), "image/jpeg"), out.timings, out.latents.shape

    futs = []
    for i in range(args.warmup):
        f, _, _ = job(i)
        f.result()
    if on_gpu:
        torch.cuda.synchronize()
    comm.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    lat = []  # per job: start -> pixels on the host (the GPU part)
    done = {}  # per job: start -> result envelope encoded (what the hive waits for)
    timings = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        ts = time.perf_counter()
        f, tm, _ = job(args.warmup + i)
        f.add_done_callback(lambda _f, i=i, ts=ts: done.__setitem__(i, time.perf_counter() - ts))
        futs.append(f)
        if on_gpu:
            torch.cuda.synchronize()
        lat.append(time.perf_counter() - ts)
        timings.append(tm)
    for f in futs:
        f.result()
    if on_gpu:
        torch.cuda.synchronize()
    comm.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    elapsed = comm.max_over_ranks(mine)
    per_rank = [mine]
    if comm.is_dist():
        per_rank = [None] * world
        torch.distributed.all_gather_object(per_rank, mine)
    p50_gpu = comm.max_over_ranks(statistics.median(lat))
    while len(done) < len(futs):  # done-callbacks run on the pool's reader thread
        time.sleep(0.001)
    p50 = comm.max_over_ranks(statistics.median(done.values()))

    images = args.batch * args.steps * world
    ips = images / elapsed
    if rank == 0:
        phase = {k: round(1000 * statistics.median([t[k] for t in timings]), 2) for k in timings[0]}
        rec = {
            "metric": CONFIGS[args.config][4],
            "value": round(ips, 4),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic prompts, random-init weights (no checkpoints offline)",
            "config": {
                "model": (CONFIGS[args.config][5] if args.family == CONFIGS[args.config][0]
                          else f"{args.family} (not the {args.config} config)"),
                "bench_config": args.config,
                "global_batch": args.batch * world,
                "seq_len": (args.res // 8) ** 2,
                "parallelism": f"dp{world}",
                "resolution": f"{args.res}x{args.res}",
                "denoise_steps": args.denoise_steps,
                "scheduler": "DPMSolverMultistepScheduler (karras)",
                "guidance_scale": args.guidance,
                "impl": args.impl,
                "hip_graphs": (not args.no_graphs) and args.impl == "hip",
            },
            "p50_job_latency_ms": round(1000 * p50, 1),
            "p50_job_latency_note": "job start -> result envelope (JPEG/base64/sha256) done",
            "p50_gpu_latency_ms": round(1000 * p50_gpu, 1),
            "world_size": world,
            "ms_per_step_per_rank": [round(1000 * t / args.steps, 2) for t in per_rank],
            "dist_backend": torch.distributed.get_backend() if comm.is_dist() else None,
            "phase_ms_median": phase,
            "model_load_s": round(load_s, 2),
            "model_load_read_s": round(load_read_s, 3),
            "model_load_all_gather_s": round(load_gather_s, 3),
            "load_bytes_read_per_rank": load_bytes,
            "model_load_read_GBps": round(load_bytes / max(load_read_s, 1e-9) / 1e9, 2),
            "load_path": (f"safetensors dir -> native sharded byte-range reads (csrc/host/csk_io.cpp) + "
                          f"{'RCCL' if on_gpu else 'gloo'} all_gather of the raw bytes" if world > 1 else
                          "safetensors dir -> native threaded pread + pinned-ring H2D (csrc/host/csk_io.cpp)"),
        }
        print(json.dumps(rec), flush=True)
    pool.shutdown()
    if comm.is_dist():
        torch.distributed.destroy_process_group()


def load_through_checkpoint(pipe, rank, world):
    """Write the pipeline's weights once as safetensors (rank 0, /dev/shm), then
    load them on every rank through models/weights.load_component inside
    ``collective_loading`` (sharded reads + all_gather with N > 1).  Returns
    (seconds, bytes this rank read from the files, read seconds, all_gather
    seconds) — the last two max over ranks, 0 for the all_gather without one."""
    import shutil
    import tempfile

    from safetensors.torch import save_file

    from chiaswarm_amd.models.layers import prepare_model
    from chiaswarm_amd.models.weights import _VAE_RENAMES, load_component
    from chiaswarm_amd.parallel import comm, sharded

    parts = [("unet", pipe.unet, None), ("vae", pipe.vae, _VAE_RENAMES)] + \
        [("text_encoder" if i == 0 else f"text_encoder_{i + 1}", m, None) for i, m in enumerate(pipe.text_encoders)]
    base = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    root = os.path.join(base, f"chiaswarm_bench_{os.getuid()}_{os.environ.get('MASTER_PORT', os.getpid())}")
    if os.environ.get("SDAAS_BENCH_FAIL_RANK") == str(rank):  # test hook: a rank dying during the load
        raise SystemExit(f"bench: rank {rank} failing on purpose (SDAAS_BENCH_FAIL_RANK)")
    if rank == 0:
        for sub, m, _ in parts:
            os.makedirs(os.path.join(root, sub), exist_ok=True)
            save_file({k: v.detach().contiguous().cpu() for k, v in m.state_dict().items()},
                      os.path.join(root, sub, "model.safetensors"))
    comm.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    nbytes = 0
    read_s = gather_s = 0.0
    with comm.collective_loading():
        for sub, m, ren in parts:
            t1 = time.perf_counter()
            load_component(m, root, sub, ren)
            if comm.collective_load_active() and sharded.LAST_READER is not None:
                nbytes += sharded.LAST_READER.read_bytes
                read_s += sharded.LAST_READER.read_s
                gather_s += sharded.LAST_READER.gather_s
            else:
                read_s += time.perf_counter() - t1
            if not (comm.collective_load_active() and sharded.LAST_READER is not None):
                nbytes += sum(os.path.getsize(f) for f in sharded.safetensors_files(os.path.join(root, sub)))
            prepare_model(m)  # re-pack for the kernels (fused QKV, NHWC conv weights ...)
    pipe.invalidate_graphs()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    load_s = comm.max_over_ranks(time.perf_counter() - t0)
    read_s, gather_s = comm.max_over_ranks(read_s), comm.max_over_ranks(gather_s)
    comm.barrier()
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    return load_s, nbytes, read_s, gather_s


if __name__ == "__main__":
    sys.exit(main())
