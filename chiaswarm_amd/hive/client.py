"""Hive protocol client (HTTP/JSON pull model, bearer token) — byte-compatible
with the reference (swarm/worker.py:58-110, :145-163; swarm/initialize.py:97-116):

  GET  {uri}/api/work?worker_version=&worker_name=   (10 s timeout)
       200 {"jobs": [...]}  -> sleep 1 s if any job else 11 s
       400 {"message": ...} -> "bad worker": raise -> 121 s backoff
       other                -> raise -> 121 s backoff
  POST {uri}/api/results  JSON body (60 s timeout)
  GET  {uri}/api/models   (no auth, 10 s)

Added: bounded retry with jitter for result submission (the
reference dropped a result on any POST exception).
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
from datetime import datetime

import aiohttp

from .. import __version__

POLL_FOUND, POLL_IDLE, POLL_ERROR = 1, 11, 121


def headers(token: str) -> dict:
    return {"Content-type": "application/json", "Authorization": f"Bearer {token}",
            "user-agent": f"chiaSWARM.worker/{__version__}"}


class HiveClient:
    def __init__(self, settings, submit_retries: int = 3, retry_base_s: float = 2.0):
        self.settings = settings
        self.api = f"{settings.sdaas_uri.rstrip('/')}/api"
        self.submit_retries = submit_retries
        self.retry_base_s = retry_base_s

    async def ask_for_work(self):
        """Returns (jobs, sleep_seconds)."""
        print(f"{datetime.now()}: Asking for work from the hive at {self.api}...")
        try:
            timeout = aiohttp.ClientTimeout(total=10)
            async with aiohttp.ClientSession(timeout=timeout) as session:
                async with session.get(f"{self.api}/work",
                                       params={"worker_version": __version__,
                                               "worker_name": self.settings.worker_name},
                                       headers=headers(self.settings.sdaas_token)) as resp:
                    if resp.status == 200:
                        body = await resp.json()
                        jobs = list(body.get("jobs", []))
                        for job in jobs:
                            print(f"Got job {job.get('id')}")
                        return jobs, (POLL_FOUND if jobs else POLL_IDLE)
                    if resp.status == 400:
                        body = await resp.json()
                        print(f"{self.api} says {body.get('message', 'bad worker')}")
                    else:
                        print(f"{self.api} returned {resp.status}")
                    resp.raise_for_status()
        except Exception as e:
            logging.exception(e)
            print(e)
            return [], POLL_ERROR
        return [], POLL_IDLE

    async def submit_result(self, result: dict) -> dict | None:
        body = json.dumps(result)
        for attempt in range(self.submit_retries + 1):
            try:
                timeout = aiohttp.ClientTimeout(total=60)
                async with aiohttp.ClientSession(timeout=timeout) as session:
                    async with session.post(f"{self.api}/results", data=body,
                                            headers=headers(self.settings.sdaas_token)) as resp:
                        if resp.status == 500:
                            print(f"The hive returned an error: {resp.reason}")
                            return None
                        if resp.status >= 400:
                            raise aiohttp.ClientResponseError(resp.request_info, resp.history, status=resp.status)
                        out = await resp.json()
                        print(f"Result {out}")
                        return out
            except Exception as e:
                logging.exception(e)
                if attempt == self.submit_retries:
                    print(f"result_worker gave up on {result.get('id')}: {e}")
                    return None
                await asyncio.sleep(self.retry_base_s * (2 ** attempt) * (0.5 + random.random()))
        return None

    def get_models(self) -> list:
        import requests

        from ..settings import save_file

        hive_uri = f"{self.settings.sdaas_uri.rstrip('/')}/"
        print(f"Fetching known model list from the hive at {hive_uri}...")
        try:
            r = requests.get(f"{hive_uri}api/models", timeout=10,
                             headers={"user-agent": f"chiaSWARM.worker/{__version__}"})
            data = r.json()
            save_file(data, "models.json")
            return data["language_models"] + data["models"]
        except Exception as e:
            print(f"Failed to fetch known model list from {hive_uri}: {e}")
            return []
