"""Job execution + error envelope (reference: swarm/generator.py:12-95).

Error classes (hive-visible):
  (a) anything raised while normalising/routing the job -> ``fatal_error: true``;
  (b) ``ValueError`` during generation (e.g. incompatible LoRA)  -> fatal;
  (c) any other exception -> non-fatal (the hive may retry elsewhere).
Image content types render the error message into a 512x512 image, others
return a text artifact; ``pipeline_config = {"error": msg}``.
"""
from __future__ import annotations

import asyncio
import logging
import time

from .. import __version__
from ..jobs.router import format_args
from ..log_setup import log_job
from ..output.processor import image_from_text, image_to_buffer, make_result, make_text_result
from ..utils.trace import trace_range


async def do_work(job, device):
    loop = asyncio.get_running_loop()
    return await loop.run_in_executor(None, synchronous_do_work_function, job, device)


def _error_result(job_id, e, content_type, fatal):
    if content_type.startswith("image/"):
        artifacts, cfg = exception_image(e, content_type)
    else:
        artifacts, cfg = exception_message(e)
    out = {"id": job_id, "artifacts": artifacts, "nsfw": cfg.get("nsfw", False),
           "worker_version": __version__, "pipeline_config": cfg}
    if fatal:
        out["fatal_error"] = True
    return out


def synchronous_do_work_function(job, device):
    job = dict(job)
    job_id = job.pop("id")
    print(f"Processing {job_id} on {device.descriptor()}")
    content_type = job.get("content_type", "image/jpeg")
    t0 = time.perf_counter()
    rec = {"id": job_id, "workflow": job.get("workflow", "txt2img"), "model": job.get("model_name"),
           "device": device.descriptor(), "images": job.get("num_images_per_prompt", 1)}

    def done(status, cfg=None, err=None):
        rec.update(status=status, seconds=round(time.perf_counter() - t0, 4))
        if err is not None:
            rec["error"] = str(err)[:300]
        if cfg:
            for k in ("seed", "timings", "batched_with", "split", "weights"):
                if k in cfg:
                    rec[k] = cfg[k]
        log_job(rec)  # one structured JSON line per job

    try:
        worker_function, kwargs = format_args(job)
    except Exception as e:  # (a) fatal: bad input
        logging.exception(e)
        done("fatal", err=e)
        return _error_result(job_id, e, content_type, True)
    try:
        t_dev = time.perf_counter()
        with trace_range(f"job {job_id}"):
            artifacts, pipeline_config = device(worker_function, **kwargs)
    except ValueError as e:  # (b) fatal
        logging.exception(e)
        done("fatal", err=e)
        return _error_result(job_id, e, content_type, True)
    except Exception as e:  # (c) retryable
        logging.exception(e)
        done("error", err=e)
        return _error_result(job_id, e, content_type, False)
    if isinstance(pipeline_config.get("timings"), dict):  # only with SDAAS_TIMINGS=1
        pipeline_config["timings"]["route"] = round(t_dev - t0, 4)
        pipeline_config["timings"]["total"] = round(time.perf_counter() - t0, 4)
    done("ok", pipeline_config)
    return {"id": job_id, "artifacts": artifacts, "nsfw": pipeline_config.get("nsfw", False),
            "worker_version": __version__, "pipeline_config": pipeline_config}


def _message(e) -> str:
    return e.args[0] if len(e.args) > 0 else "error generating image"


def exception_image(e, content_type):
    message = _message(e)
    img = image_from_text(str(message))
    return {"primary": make_result(image_to_buffer(img, content_type), img, content_type)}, {"error": message}


def exception_message(e):
    return {"primary": make_text_result(str(e))}, {"error": _message(e)}
