"""bench.py's multi-rank contract on CPU: ``--gpus 2`` without torchrun env
vars spawns two rank processes (gloo), every rank runs its own job, and rank 0
prints ONE JSON line whose ``n_gpus`` / ``world_size`` is the rank count and
whose images/s aggregates over both ranks."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_spawns_ranks_cpu():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--family", "tiny", "--steps", "2", "--warmup", "1", "--denoise-steps", "2", "--res", "64",
                        "--batch", "1"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["dist_backend"] == "gloo"
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 2
    # value = images of BOTH ranks over the max-over-ranks wall time
    assert abs(rec["value"] - 2 * rec["steps"] / (rec["ms_per_step"] * rec["steps"] / 1000)) < 0.05 * rec["value"]
    assert rec["p50_job_latency_ms"] >= rec["p50_gpu_latency_ms"]


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--family", "tiny", "--steps", "1", "--warmup", "0", "--denoise-steps", "1", "--res", "64",
                        "--batch", "1"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_failing_rank_ends_the_run_fast():
    """A rank that dies during the model load (the others block in its
    collective) ends the whole run within seconds, non-zero, naming the rank —
    not after the 600 s process-group timeout."""
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["SDAAS_BENCH_FAIL_RANK"] = "1"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--family", "tiny", "--steps", "1", "--warmup", "0", "--denoise-steps", "1", "--res", "64",
                        "--batch", "1"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    took = time.monotonic() - t0
    assert r.returncode != 0
    # (gloo drops rank 0 too when its peer's socket closes; RCCL would leave it
    # blocked in the collective until the poll terminates it)
    assert "failing on purpose" in r.stderr
    assert took < 60, took  # two interpreter + torch start-ups, then the poll notices at once


def test_sdxl_config_two_ranks_cpu():
    """``--config sdxl`` (BASELINE config #3: SDXL-base 1024², 30 steps, one
    image per rank) labels its metric / model; here on the tiny SDXL-structured
    family (text_time add-embedding, two text encoders) over 2 gloo ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "sdxl", "--family", "tiny-xl",
                        "--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1", "--denoise-steps", "2",
                        "--res", "64"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert "SDXL-base 1024×1024 30-step" in rec["metric"] and rec["config"]["bench_config"] == "sdxl"
    assert rec["config"]["global_batch"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert len(rec["ms_per_step_per_rank"]) == 2 and max(rec["ms_per_step_per_rank"]) <= rec["ms_per_step"] + 1e-6
    assert rec["model_load_read_s"] >= 0 and rec["model_load_all_gather_s"] > 0


def test_bench_through_supervisor_cpu(tmp_path):
    """``--through-supervisor``: the jobs go fake hive ->
    Supervisor -> ProcessExecutor child -> router -> pipeline -> envelope ->
    POST, and the JSON line reports the serving path's images/s and p50."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["SDAAS_ROOT"] = str(tmp_path)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--through-supervisor", "--device", "cpu",
                        "--family", "tiny", "--steps", "3", "--warmup", "1", "--denoise-steps", "2", "--res", "64",
                        "--batch", "2"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["value"] > 0 and rec["p50_job_latency_ms"] > 0
    assert "Supervisor" in rec["path"] and rec["config"]["global_batch"] == 2


def test_bench_under_torchrun_cpu():
    """The driver's launch form: ``python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus
    N ...`` — ranks come from torchrun's env, rank 0 prints the one line."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--device", "cpu", "--family", "tiny", "--steps", "2", "--warmup", "1", "--denoise-steps", "2",
                        "--res", "64", "--batch", "1"], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == "dp2" and len(rec["ms_per_step_per_rank"]) == 2
