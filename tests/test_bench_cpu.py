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
