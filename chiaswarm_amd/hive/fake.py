"""In-process fake hive (aiohttp) with injectable faults, plus a tiny static
file server for start_image_uri / video_uri / stitch inputs.
Serves the hive protocol of swarm/worker.py:58-163 (GET /api/work, POST
/api/results, GET /api/models): used by the tests and by
``bench.py --through-supervisor`` (the serving path end to end)."""
from __future__ import annotations

import asyncio
import io
import json
import threading
import time

from aiohttp import web
from PIL import Image


class FakeHive:
    def __init__(self, jobs=None, faults=None, models=None):
        self.jobs = list(jobs or [])
        self.faults = list(faults or [])  # per poll: None | 400 | 500 | "slow"
        self.result_faults = []           # per POST: None | 500 | 503
        self.results = []
        self.result_times = []  # time.monotonic() of each accepted POST
        self.polls = 0
        self.poll_params = []
        self.auth = []
        self.files: dict[str, tuple[bytes, str]] = {}
        self.models = models or {"language_models": [], "models": [
            {"model_name": "tiny/sd", "revision": "main", "parameters": {"can_preload": True}}]}
        self.runner = None
        self.port = None

    async def work(self, request):
        self.polls += 1
        self.poll_params.append(dict(request.query))
        self.auth.append(request.headers.get("Authorization"))
        fault = self.faults.pop(0) if self.faults else None
        if fault == 400:
            return web.json_response({"message": "slow results"}, status=400)
        if fault == 500:
            return web.Response(status=500)
        jobs, self.jobs = self.jobs, []
        return web.json_response({"jobs": jobs})

    async def post_results(self, request):
        fault = self.result_faults.pop(0) if self.result_faults else None
        if fault == 503:
            return web.Response(status=503)
        body = await request.json()
        if fault == 500:
            return web.Response(status=500)
        self.results.append(body)
        self.result_times.append(time.monotonic())
        return web.json_response({"ok": True, "id": body.get("id")})

    async def get_models(self, request):
        return web.json_response(self.models)

    async def get_file(self, request):
        name = request.match_info["name"]
        if name not in self.files:
            return web.Response(status=404)
        data, ctype = self.files[name]
        return web.Response(body=data, content_type=ctype.split(";")[0])

    def add_image(self, name, size=(96, 64), color=(200, 30, 30), fmt="PNG"):
        buf = io.BytesIO()
        Image.new("RGB", size, color).save(buf, format=fmt)
        self.files[name] = (buf.getvalue(), "image/png" if fmt == "PNG" else "image/jpeg")
        return f"{self.base}/files/{name}"

    def add_file(self, name, data: bytes, ctype: str):
        self.files[name] = (data, ctype)
        return f"{self.base}/files/{name}"

    @property
    def base(self):
        return f"http://127.0.0.1:{self.port}"

    def start(self):
        """Run the server on a background thread's event loop."""
        ready = threading.Event()

        def run():
            self.loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self.loop)
            app = web.Application(client_max_size=64 << 20)
            app.router.add_get("/api/work", self.work)
            app.router.add_post("/api/results", self.post_results)
            app.router.add_get("/api/models", self.get_models)
            app.router.add_get("/files/{name}", self.get_file)
            self.runner = web.AppRunner(app)
            self.loop.run_until_complete(self.runner.setup())
            site = web.TCPSite(self.runner, "127.0.0.1", 0)
            self.loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            ready.set()
            self.loop.run_forever()

        self.thread = threading.Thread(target=run, daemon=True)
        self.thread.start()
        if not ready.wait(10):
            raise RuntimeError("fake hive failed to start")
        return self

    def stop(self):
        async def _down():
            await self.runner.cleanup()

        fut = asyncio.run_coroutine_threadsafe(_down(), self.loop)
        fut.result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)


def dumps(x):
    return json.dumps(x)
