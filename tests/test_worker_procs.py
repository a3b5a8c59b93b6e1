"""The multi-process worker on CPU (reference behaviour: swarm/worker.py:40-44
one worker per GPU, :113-128 device_worker): per-device child processes
("cpu" children here, GPU children on the box), the watchdog, the node
process group (gloo here, RCCL over xGMI on the GPU node), collective sharded
preload, and multi-image jobs split across children.

* a child that dies in the middle of a job -> non-fatal error envelope for that
  job, a fresh child that runs the next job;
* a child that hangs past the job timeout -> same;
* two children form a gloo group, preload a model with sharded reads, and a
  3-image txt2img job split over both returns the images the unsplit job does.
"""
import asyncio
import base64
import io
import os

import numpy as np
import pytest
from PIL import Image

from chiaswarm_amd.runtime.worker import ProcessExecutor, Supervisor, ThreadExecutor, _ranges, group_envs
from chiaswarm_amd.settings import Settings
from tests.fakehive import FakeHive

TINY = {"model_name": "tiny/sd", "prompt": "a red fox", "num_inference_steps": 2, "height": 64, "width": 64}


@pytest.fixture(autouse=True)
def sdaas_root(tmp_path, monkeypatch):
    from chiaswarm_amd.runtime import model_cache

    # the in-process model cache is per process: a "tiny/sd" pipeline another test
    # left in it (other weights, other SDAAS_ROOT) must not serve this test's jobs
    monkeypatch.setattr(model_cache, "_CACHE", None)
    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    monkeypatch.setenv("CSK_TEST_HOOKS", "1")  # inherited by spawned children
    return tmp_path


def _img(result):
    return np.asarray(Image.open(io.BytesIO(base64.b64decode(result["artifacts"]["primary"]["blob"]))).convert("RGB"),
                      dtype=np.int16)


def test_ranges_cover_all_images():
    assert _ranges(5, 2) == [(0, 3), (3, 5)]
    assert _ranges(4, 4) == [(0, 1), (1, 2), (2, 3), (3, 4)]


def test_process_executor_recovers_from_crash_and_hang():
    ex = ProcessExecutor("cpu", job_timeout_s=120)  # generous: a loaded box slows child start-up
    try:
        async def main():
            crashed = await ex.run({"id": "c1", **TINY, "_test": "exit"})
            ok1 = await ex.run({"id": "ok1", **TINY, "seed": 3})
            ex.job_timeout_s = 4
            hung = await ex.run({"id": "h1", **TINY, "_test": "hang"})
            ex.job_timeout_s = 120
            ok2 = await ex.run({"id": "ok2", **TINY, "seed": 3})
            return crashed, ok1, hung, ok2

        crashed, ok1, hung, ok2 = asyncio.run(main())
        assert crashed["id"] == "c1" and "fatal_error" not in crashed
        assert "crashed" in crashed["pipeline_config"]["error"]
        assert hung["id"] == "h1" and "fatal_error" not in hung and "timed out" in hung["pipeline_config"]["error"]
        assert ex.restarts == 2
        for r in (ok1, ok2):
            assert "error" not in r["pipeline_config"], r["pipeline_config"]
        assert np.array_equal(_img(ok1), _img(ok2))  # fresh children reproduce the seed
    finally:
        ex.close()


def test_child_owns_encoder_processes_and_dies_with_its_parent(tmp_path):
    """The device child is not daemonic, so it can start its JPEG encoder
    PROCESSES (a daemonic child fell back to encoding on its GPU thread); its
    envelopes come back encoded, and an orphaned child exits by itself."""
    import subprocess
    import sys
    import time

    ex = ProcessExecutor("cpu", env={"CSK_CHILD_ENCODERS": "1"}, job_timeout_s=120)
    try:
        r = asyncio.run(ex.run({"id": "e1", **TINY, "seed": 3}))
        assert ex.ready.wait(60) and ex.encoders == "process"
        assert "error" not in r["pipeline_config"] and _img(r).shape == (64, 64, 3)
    finally:
        ex.close()
    # orphan: a parent that starts an executor and is SIGKILLed; its child must follow
    pidfile = tmp_path / "child.pid"
    code = ("import sys, time, os; sys.path.insert(0, %r)\n"
            "from chiaswarm_amd.runtime.worker import ProcessExecutor\n"
            "ex = ProcessExecutor('cpu')\n"
            "assert ex.ready.wait(120)\n"
            "open(%r, 'w').write(str(ex.proc.pid))\n"
            "time.sleep(600)\n") % (os.getcwd(), str(pidfile))
    parent = subprocess.Popen([sys.executable, "-c", code])
    try:
        for _ in range(300):
            if pidfile.exists() and pidfile.read_text():
                break
            time.sleep(0.5)
        child = int(pidfile.read_text())
    finally:
        parent.kill()
        parent.wait()
    for _ in range(40):  # the watchdog polls once a second
        try:
            os.kill(child, 0)
        except ProcessLookupError:
            break
        time.sleep(0.5)
    else:
        os.kill(child, 9)
        raise AssertionError("orphaned device child kept running")


def _save_tiny_model(root):
    """A diffusers-layout tiny checkpoint under $SDAAS_ROOT/models/tiny/sd."""
    from safetensors.torch import save_file

    from chiaswarm_amd.pipelines.sd import StableDiffusion

    pipe = StableDiffusion("tiny", device="cpu", seed=77)
    d = root / "models" / "tiny" / "sd"
    for sub, m in (("unet", pipe.unet), ("vae", pipe.vae), ("text_encoder", pipe.text_encoders[0])):
        os.makedirs(d / sub, exist_ok=True)
        save_file({k: v.contiguous() for k, v in m.state_dict().items()}, str(d / sub / "model.safetensors"))
    from tests.test_checkpoints import _train_bpe

    _train_bpe(str(d / "tokenizer"))  # real weights need their tokenizer (strict loads)
    return d


def test_group_preload_and_split_job_matches_unsplit(sdaas_root):
    _save_tiny_model(sdaas_root)
    job = {"id": "multi", **TINY, "seed": 1234, "num_images_per_prompt": 3, "content_type": "image/png"}
    # unsplit reference: one in-process executor
    solo_hive = FakeHive(jobs=[dict(job)]).start()
    try:
        s = Settings()
        s.sdaas_uri, s.sdaas_token = solo_hive.base, "t"

        async def solo():
            sup = Supervisor(s, executors=[ThreadExecutor("cpu")], hive=None)
            await sup.run(max_polls=1)

        asyncio.run(solo())
        ref = solo_hive.results[0]
    finally:
        solo_hive.stop()
    assert ref["pipeline_config"].get("split") is None
    assert ref["pipeline_config"]["weights"].endswith(os.path.join("tiny", "sd"))

    hive = FakeHive(jobs=[dict(job)]).start()
    envs = group_envs(2)
    exs = [ProcessExecutor("cpu", env=e) for e in envs]
    try:
        s = Settings()
        s.sdaas_uri, s.sdaas_token = hive.base, "t"
        s.preload = "tiny/sd"
        s.max_batch = 1

        async def main():
            sup = Supervisor(s, executors=exs)
            await sup.run(max_polls=1)
            return sup

        sup = asyncio.run(main())
        assert all(e.ready.wait(5) for e in exs)
        assert all("gloo rank" in e.ready_info for e in exs), [e.ready_info for e in exs]
        assert sup.group_ok() and sup.store is not None  # the rendezvous lives in the supervisor
        assert sup.splits == 1
        res = hive.results[0]
        assert res["id"] == "multi" and res["pipeline_config"]["split"] == 2
        assert res["pipeline_config"]["seed"] == 1234
        assert res["pipeline_config"]["weights"].endswith(os.path.join("tiny", "sd"))
        a, b = _img(res), _img(ref)
        assert a.shape == b.shape
        d = np.abs(a - b)
        assert d.mean() < 0.5 and d.max() <= 24  # same seeds per image; only batch-size summation order differs
    finally:
        hive.stop()
        for e in exs:
            e.close()


def test_rank0_crash_survivors_restart_and_regroup(sdaas_root):
    """World 3 (gloo): rank 0's child dies in the middle of a job.  The store is
    the supervisor's, so the survivors keep serving; the restarted child serves
    rank-local; the idle supervisor re-forms the group (generation 1) and a
    split job then runs over it again (images sent rank-to-rank)."""
    _save_tiny_model(sdaas_root)
    exs = [ProcessExecutor("cpu", env=e, job_timeout_s=300) for e in group_envs(3)]
    try:
        s = Settings()
        s.max_batch = 1

        async def main():
            sup = Supervisor(s, executors=exs, hive=FakeHive(jobs=[]))
            for e in exs:
                await asyncio.get_running_loop().run_in_executor(None, e.ready.wait, 120)
            assert sup.group_ok()
            crashed = await exs[0].run({"id": "c", **TINY, "_test": "exit"})
            assert "crashed" in crashed["pipeline_config"]["error"] and exs[0].restarts == 1
            await asyncio.get_running_loop().run_in_executor(None, exs[0].ready.wait, 120)
            assert not sup.group_ok()  # the fresh child is rank-local: no collectives now
            later = await asyncio.gather(*(e.run({"id": f"j{i}", **TINY, "seed": 5}) for i, e in enumerate(exs)))
            for r in later:
                assert "error" not in r["pipeline_config"], r["pipeline_config"]
            imgs = [_img(r) for r in later]
            assert all(np.array_equal(imgs[0], im) for im in imgs[1:])
            assert await sup.regroup()
            assert all(e.group["gen"] == 1 for e in exs)
            job = {"id": "multi", **TINY, "seed": 99, "num_images_per_prompt": 3, "content_type": "image/png"}
            res = await sup._run_split(job, list(exs))
            return sup, res

        sup, res = asyncio.run(main())
        assert sup.splits == 1 and res["id"] == "multi"
        assert res["pipeline_config"]["split"] == 3 and res["pipeline_config"]["seed"] == 99
        assert _img(res).shape[:2] == (128, 128)  # 3 images -> 2x2 grid of 64x64
    finally:
        for e in exs:
            e.close()


def test_rank_dying_mid_preload_does_not_wedge_the_node(sdaas_root):
    """A child that dies inside a collective preload: the supervisor kills any
    peer still blocked in the all_gather, reports the preload as failed within
    seconds (not after the 3600 s preload timeout), and every child serves jobs."""
    import time

    _save_tiny_model(sdaas_root)
    exs = [ProcessExecutor("cpu", env=e, job_timeout_s=300) for e in group_envs(2)]
    try:
        s = Settings()
        s.max_batch = 1

        async def main():
            sup = Supervisor(s, executors=exs, hive=FakeHive(jobs=[]))
            for e in exs:
                await asyncio.get_running_loop().run_in_executor(None, e.ready.wait, 120)
            t0 = time.monotonic()
            with pytest.raises(RuntimeError, match="preload failed"):
                await sup.preload(["__test_exit__", "tiny/sd"])
            dt = time.monotonic() - t0
            return dt, await asyncio.gather(*(e.run({"id": f"p{i}", **TINY, "seed": 2}) for i, e in enumerate(exs)))

        dt, res = asyncio.run(main())
        assert dt < 120
        # the dead rank is restarted; its peer was either killed out of the wedged
        # all_gather (restarted too) or saw the broken group itself and returned
        assert exs[1].restarts == 1
        for r in res:
            assert "error" not in r["pipeline_config"], r["pipeline_config"]
    finally:
        for e in exs:
            e.close()
