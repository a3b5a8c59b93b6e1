"""Stress of the per-device process layer (SURVEY §5.2 race detection, §5.3
failure detection): many jobs through two child processes with injected
crashes; every job must come back exactly once with its own id, crashed jobs
as non-fatal errors, the rest as successes, and nothing may deadlock."""
import asyncio
import random

import pytest

from chiaswarm_amd.runtime.worker import ProcessExecutor, Supervisor
from chiaswarm_amd.settings import Settings
from tests.fakehive import FakeHive

TINY = {"model_name": "tiny/sd", "prompt": "p", "num_inference_steps": 1, "height": 64, "width": 64}


@pytest.fixture(autouse=True)
def env(tmp_path, monkeypatch):
    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    monkeypatch.setenv("CSK_TEST_HOOKS", "1")


def test_many_jobs_with_crashes_through_two_children():
    rng = random.Random(7)
    jobs = []
    for i in range(24):
        j = {"id": f"s{i}", **TINY, "seed": i, "prompt": f"p{i}"}
        if i in (3, 11, 19):
            j["_test"] = "exit"
        if rng.random() < 0.3:
            j["num_images_per_prompt"] = 2  # some multi-image jobs (split across both children when idle)
        jobs.append(j)
    hive = FakeHive(jobs=jobs).start()
    exs = [ProcessExecutor("cpu", job_timeout_s=120) for _ in range(2)]
    try:
        s = Settings()
        s.sdaas_uri, s.sdaas_token = hive.base, "t"
        s.max_batch = 4  # coalescing on as well

        async def main():
            sup = Supervisor(s, executors=exs)
            await asyncio.wait_for(sup.run(max_polls=1), timeout=600)
            return sup

        sup = asyncio.run(main())
        ids = [r["id"] for r in hive.results]
        assert sorted(ids) == sorted(j["id"] for j in jobs)  # each job exactly once
        by = {r["id"]: r for r in hive.results}
        ok = 0
        for j in jobs:
            r = by[j["id"]]
            err = r["pipeline_config"].get("error")
            if "_test" in j:
                assert err and "fatal_error" not in r
            elif err:  # collateral: coalesced into the same batch as a crashing job
                assert "crashed" in err and "fatal_error" not in r, err
            else:
                ok += 1
        assert ok >= 12
        assert sum(e.restarts for e in exs) >= 1
    finally:
        hive.stop()
        for e in exs:
            e.close()
