#!/usr/bin/env python
"""Fine-grained host/device timing of the pre-denoise part of an SD2.1 job
(tokenize, text encoder, cross-attention K/V, noise), each bracketed by a
device sync, to find host overhead outside the hipGraph-replayed steps."""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402


def main():
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    ops._lib.load()
    dev = torch.device("cuda", 0)
    p = StableDiffusion("sd21", device=dev, seed=0)
    prompts = ["a photograph of an astronaut riding a horse"] * 4
    negs = ["blurry"] * 4

    def t(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return r, (time.perf_counter() - t0) * 1000

    for it in range(4):
        ids, tk = t(lambda: p.tokenizers[0](negs + prompts).to(dev))
        out, te = t(lambda: p.text_encoders[0](ids))
        kv, tkv = t(lambda: p.unet.encode_context(out[0]))
        enc, tall = t(lambda: p.encode_prompt(prompts, negs, True))
        print(f"iter {it}: tokenize {tk:.2f} ms  text_encoder {te:.2f} ms  cross-kv {tkv:.2f} ms  "
              f"encode_prompt {tall:.2f} ms", flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def jobs():
    """The bench's job loop with and without the overlapped result-encoding thread."""
    import concurrent.futures as cf

    from chiaswarm_amd.output.processor import OutputProcessor
    from chiaswarm_amd.pipelines.sd import StableDiffusion
    from chiaswarm_amd.schedulers import get_scheduler

    ops._lib.load()
    dev = torch.device("cuda", 0)
    p = StableDiffusion("sd21", device=dev, seed=0)
    pool = cf.ThreadPoolExecutor(max_workers=2)
    for overlap in (False, True, False, True):
        fut = None
        for i in range(3):
            g = torch.Generator(device=dev).manual_seed(i)
            out = p(prompt="a fox", negative_prompt="blurry", num_inference_steps=50, num_images_per_prompt=4,
                    height=512, width=512, generator=g, scheduler=get_scheduler("DPMSolverMultistepScheduler"))

            def enc(images=out.images):
                op = OutputProcessor(["primary"], "image/jpeg")
                op.add_outputs(images)
                return op.get_results()

            if overlap:
                fut = pool.submit(enc)
            else:
                enc()
            print(f"overlap={overlap} job {i}: " + " ".join(f"{k} {v * 1000:.1f}" for k, v in out.timings.items()),
                  flush=True)
        if fut:
            fut.result()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "jobs":
    jobs()
