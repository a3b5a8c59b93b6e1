"""Worker plumbing on CPU: error classification, device wrapper, the full
supervisor loop against a fake hive with injected faults,
and BASELINE config #1 (txt2img through the real router/device/encoder)."""
import asyncio
import base64
import io

import pytest
from PIL import Image

from chiaswarm_amd import __version__
from chiaswarm_amd.hive.client import POLL_ERROR, POLL_FOUND, POLL_IDLE, HiveClient
from chiaswarm_amd.runtime.device import Device
from chiaswarm_amd.runtime.generator import synchronous_do_work_function
from chiaswarm_amd.runtime.worker import Supervisor, ThreadExecutor
from chiaswarm_amd.settings import Settings
from tests.fakehive import FakeHive

TINY = {"model_name": "tiny/sd", "prompt": "a red fox", "num_inference_steps": 3, "height": 64, "width": 64}


@pytest.fixture(autouse=True)
def sdaas_root(tmp_path, monkeypatch):
    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))


def test_success_envelope():
    r = synchronous_do_work_function({"id": "j1", **TINY, "seed": 42}, Device("cpu"))
    assert r["id"] == "j1" and r["worker_version"] == __version__
    assert r["nsfw"] is False and "fatal_error" not in r
    assert r["pipeline_config"]["seed"] == 42
    img = Image.open(io.BytesIO(base64.b64decode(r["artifacts"]["primary"]["blob"])))
    assert img.size == (64, 64) and img.format == "JPEG"


def test_seed_determinism_and_grid():
    job = {"id": "j", **TINY, "seed": 7, "num_images_per_prompt": 2, "content_type": "image/png"}
    a = synchronous_do_work_function(dict(job), Device("cpu"))
    b = synchronous_do_work_function(dict(job), Device("cpu"))
    assert a["artifacts"]["primary"]["sha256_hash"] == b["artifacts"]["primary"]["sha256_hash"]
    img = Image.open(io.BytesIO(base64.b64decode(a["artifacts"]["primary"]["blob"])))
    assert img.size == (128, 64) and img.format == "PNG"


def test_fatal_on_bad_arguments():
    r = synchronous_do_work_function({"id": "j2", "model_name": "m", "height": 4096, "width": 64}, Device("cpu"))
    assert r["fatal_error"] is True and "max image size" in r["pipeline_config"]["error"]
    assert r["artifacts"]["primary"]["content_type"] == "image/jpeg"


def test_fatal_on_value_error_text_artifact():
    job = {"id": "j3", **TINY, "lora": "/nonexistent/lora.safetensors", "content_type": "audio/mpeg"}
    r = synchronous_do_work_function(job, Device("cpu"))
    assert r["fatal_error"] is True
    assert r["artifacts"]["primary"]["content_type"] == "application/json"


def test_nonfatal_on_runtime_error(monkeypatch):
    from chiaswarm_amd.pipelines import diffusion

    def boom(*a, **k):
        raise RuntimeError("out of memory")

    monkeypatch.setattr(diffusion, "diffusion_callback", boom)
    r = synchronous_do_work_function({"id": "j4", **TINY}, Device("cpu"))
    assert "fatal_error" not in r and r["pipeline_config"]["error"] == "out of memory"


def test_device_busy():
    d = Device("cpu")
    d.mutex.acquire()
    with pytest.raises(Exception, match="busy"):
        d(lambda *a, **k: ({}, {}), model_name="m")


def _settings(hive):
    s = Settings()
    s.sdaas_uri = hive.base
    s.sdaas_token = "tok"
    s.worker_name = "w1"
    return s


def test_hive_client_cadence_and_faults():
    hive = FakeHive(jobs=[{"id": "a", **TINY}], faults=[None, None, 400, 500]).start()
    try:
        c = HiveClient(_settings(hive))
        jobs, sl = asyncio.run(c.ask_for_work())
        assert [j["id"] for j in jobs] == ["a"] and sl == POLL_FOUND
        assert asyncio.run(c.ask_for_work()) == ([], POLL_IDLE)
        assert asyncio.run(c.ask_for_work())[1] == POLL_ERROR  # 400 bad worker
        assert asyncio.run(c.ask_for_work())[1] == POLL_ERROR  # 500
        assert hive.auth[0] == "Bearer tok"
        assert hive.poll_params[0] == {"worker_version": __version__, "worker_name": "w1"}
    finally:
        hive.stop()


def test_submit_retry_with_backoff():
    hive = FakeHive().start()
    hive.result_faults = [503, 503]
    try:
        c = HiveClient(_settings(hive), submit_retries=3, retry_base_s=0.01)
        out = asyncio.run(c.submit_result({"id": "r1", "artifacts": {}}))
        assert out == {"ok": True, "id": "r1"} and len(hive.results) == 1
    finally:
        hive.stop()


def test_supervisor_end_to_end():
    jobs = [{"id": f"job{i}", **TINY, "seed": i} for i in range(3)]
    jobs.append({"id": "bad", "model_name": "m", "height": 9999, "width": 9})
    hive = FakeHive(jobs=jobs).start()
    try:
        async def main():
            sup = Supervisor(_settings(hive), executors=[ThreadExecutor("cpu")])
            await sup.run(max_polls=3)
            return sup

        sup = asyncio.run(main())
        ids = sorted(r["id"] for r in hive.results)
        assert ids == ["bad", "job0", "job1", "job2"]
        bad = [r for r in hive.results if r["id"] == "bad"][0]
        assert bad["fatal_error"] is True
        assert sup.results_submitted == 4
    finally:
        hive.stop()


def test_stitch_workflow():
    hive = FakeHive().start()
    try:
        urls = [hive.add_image(f"r{i}.png", size=(200, 100 + 40 * i), color=(50 * i, 80, 90)) for i in range(5)]
        job = {"id": "s", "model_name": "stitch", "workflow": "stitch",
               "jobs": [{"resultUri": u, "fileName": f"f{i}.png", "model_name": f"m{i}"} for i, u in enumerate(urls)]}
        r = synchronous_do_work_function(job, Device("cpu"))
        img = Image.open(io.BytesIO(base64.b64decode(r["artifacts"]["primary"]["blob"])))
        assert img.size == (144 * 3, 144 * 3)
        m = r["pipeline_config"]["image_map"]
        assert len(m) == 5 and m[3]["coords"] == "0,144,144,288" and m[4]["alt"] == "m4"
        assert m[0]["filename"] == "f0.png"
    finally:
        hive.stop()


def test_batched_jobs_match_solo_results():
    """Coalesced txt2img jobs (runtime.batcher) return the images each job gets alone."""
    from chiaswarm_amd.runtime.batcher import run_jobs

    jobs = [{"id": f"b{i}", **TINY, "seed": 100 + i, "num_images_per_prompt": 1 + (i % 2),
             "prompt": f"fox {i}"} for i in range(3)]
    jobs.append({"id": "solo", **TINY, "seed": 5, "height": 128})  # different size: not coalesced
    jobs.append({"id": "bad", "model_name": "m", "height": 9999, "width": 9})
    dev = Device("cpu")
    batched = run_jobs([dict(j) for j in jobs], dev, max_images=8)
    assert [r["id"] for r in batched] == [j["id"] for j in jobs]
    assert batched[0]["pipeline_config"].get("batched_with") == 3
    assert batched[-1]["fatal_error"] is True
    for j, r in zip(jobs[:4], batched[:4]):
        solo = synchronous_do_work_function(dict(j), dev)
        assert r["pipeline_config"]["seed"] == solo["pipeline_config"]["seed"]
        a = Image.open(io.BytesIO(base64.b64decode(r["artifacts"]["primary"]["blob"]))).convert("RGB")
        b = Image.open(io.BytesIO(base64.b64decode(solo["artifacts"]["primary"]["blob"]))).convert("RGB")
        assert a.size == b.size
        import numpy as np

        d = np.abs(np.asarray(a, np.int16) - np.asarray(b, np.int16))
        # same noise, same sampler: only fp32 summation-order differences of the larger batch remain
        assert d.mean() < 0.5 and d.max() <= 24


def test_supervisor_coalesces_queued_jobs():
    jobs = [{"id": f"q{i}", **TINY, "seed": i} for i in range(4)]
    hive = FakeHive(jobs=jobs).start()
    try:
        async def main():
            s = _settings(hive)
            s.max_batch = 4
            sup = Supervisor(s, executors=[ThreadExecutor("cpu")])
            await sup.run(max_polls=2)
            return sup

        asyncio.run(main())
        assert sorted(r["id"] for r in hive.results) == [f"q{i}" for i in range(4)]
        assert any(r["pipeline_config"].get("batched_with", 1) > 1 for r in hive.results)
    finally:
        hive.stop()


def test_batched_stochastic_sampler_matches_solo():
    """Ancestral sampler: each coalesced job draws its per-step noise from its own
    generator, so its images do not depend on which jobs it was batched with."""
    import numpy as np

    from chiaswarm_amd.runtime.batcher import run_jobs

    jobs = [{"id": f"a{i}", **TINY, "parameters": {"scheduler_type": "EulerAncestralDiscreteScheduler"},
             "seed": 300 + i, "num_images_per_prompt": 1 + i,
             "prompt": f"owl {i}", "content_type": "image/png"} for i in range(2)]
    dev = Device("cpu")
    batched = run_jobs([dict(j) for j in jobs], dev, max_images=8)
    assert batched[0]["pipeline_config"].get("batched_with") == 2
    for j, r in zip(jobs, batched):
        solo = synchronous_do_work_function(dict(j), dev)
        a = np.asarray(Image.open(io.BytesIO(base64.b64decode(r["artifacts"]["primary"]["blob"]))), np.int16)
        b = np.asarray(Image.open(io.BytesIO(base64.b64decode(solo["artifacts"]["primary"]["blob"]))), np.int16)
        d = np.abs(a - b)
        assert d.mean() < 0.5 and d.max() <= 24


def test_every_job_writes_a_structured_log_line(caplog):
    import json
    import logging

    with caplog.at_level(logging.INFO, logger="chiaswarm_amd.jobs"):
        synchronous_do_work_function({"id": "L1", **TINY, "seed": 9}, Device("cpu"))
        synchronous_do_work_function({"id": "L2", "model_name": "m", "height": 9999, "width": 9}, Device("cpu"))
    recs = [json.loads(r.getMessage()) for r in caplog.records if r.name == "chiaswarm_amd.jobs"]
    assert [r["id"] for r in recs] == ["L1", "L2"]
    assert recs[0]["status"] == "ok" and recs[0]["seed"] == 9 and recs[0]["seconds"] > 0
    assert recs[1]["status"] == "fatal" and "error" in recs[1]


def test_batched_ddim_eta_matches_solo_and_splits_by_eta():
    """eta is part of the batch key and reaches the batched sampler: a DDIM
    eta > 0 job gives its solo images when coalesced."""
    import numpy as np

    from chiaswarm_amd.runtime.batcher import run_jobs

    base = {**TINY, "parameters": {"scheduler_type": "DDIMScheduler"}, "content_type": "image/png"}
    jobs = [{"id": f"e{i}", **base, "seed": 40 + i, "eta": 1.0} for i in range(2)]
    jobs.append({"id": "e0eta", **base, "seed": 50})  # eta 0: not coalesced with the eta 1 jobs
    dev = Device("cpu")
    batched = run_jobs([dict(j) for j in jobs], dev, max_images=8)
    assert batched[0]["pipeline_config"].get("batched_with") == 2
    assert batched[2]["pipeline_config"].get("batched_with", 1) == 1
    for j, r in zip(jobs[:2], batched[:2]):
        solo = synchronous_do_work_function(dict(j), dev)
        a = np.asarray(Image.open(io.BytesIO(base64.b64decode(r["artifacts"]["primary"]["blob"]))), np.int16)
        b = np.asarray(Image.open(io.BytesIO(base64.b64decode(solo["artifacts"]["primary"]["blob"]))), np.int16)
        d = np.abs(a - b)
        assert d.mean() < 0.5 and d.max() <= 24


def test_batched_unknown_kwarg_fails_like_solo():
    """An unknown pipeline kwarg fails the job batched exactly as it does solo
    (retryable TypeError envelope), and does not sink its batch mates."""
    from chiaswarm_amd.runtime.batcher import run_jobs

    jobs = [{"id": "k0", **TINY, "seed": 1}, {"id": "k1", **TINY, "seed": 2, "not_a_pipeline_arg": 3}]
    dev = Device("cpu")
    out = run_jobs([dict(j) for j in jobs], dev, max_images=8)
    solo = synchronous_do_work_function(dict(jobs[1]), dev)
    assert "error" not in out[0]["pipeline_config"]
    assert "not_a_pipeline_arg" in out[1]["pipeline_config"]["error"]
    assert out[1]["pipeline_config"]["error"] == solo["pipeline_config"]["error"]
    assert "fatal_error" not in out[1]


def test_restart_fails_every_pending_job():
    """A child restart (e.g. a regroup that timed out) resolves the futures of
    jobs already sent to it, not only control messages."""
    from chiaswarm_amd.runtime.worker import ProcessExecutor

    class _Proc:
        def kill(self):
            pass

        def join(self, timeout=None):
            pass

    async def main():
        ex = ProcessExecutor.__new__(ProcessExecutor)
        ex.loop = asyncio.get_running_loop()
        ex.pending = {"job-1": ex.loop.create_future(), "__regrouped__": ex.loop.create_future()}
        ex.proc, ex.env, ex.restarts = _Proc(), {}, 0
        ex._start = lambda: None
        futs = dict(ex.pending)
        ex._restart()
        await asyncio.sleep(0)
        return {k: f.result() for k, f in futs.items()}, ex.pending

    res, left = asyncio.run(main())
    assert res == {"job-1": (None, "GPU worker restarted"), "__regrouped__": (None, "GPU worker restarted")}
    assert left == {}
