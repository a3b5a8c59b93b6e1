#!/usr/bin/env python
"""Fine-grained host/device timing of the pre-denoise part of an SD2.1 job
(tokenize, text encoder, cross-attention K/V, noise), each bracketed by a
device sync, to find host overhead outside the hipGraph-replayed steps."""
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


if __name__ == "__main__":
    main()
