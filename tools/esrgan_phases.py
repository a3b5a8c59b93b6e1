import os, time, statistics
os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1"); os.environ.setdefault("SDAAS_OFFLINE", "1")
import sys; sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from PIL import Image
from chiaswarm_amd.pipelines.esrgan import load_esrgan, upscale_x4, _run_u8
if len(sys.argv) > 1:  # run another pipeline first (python tools/esrgan_phases.py sdxl): the multi-config bench order
    from chiaswarm_amd.pipelines.sd import StableDiffusion
    p = StableDiffusion(sys.argv[1], device=torch.device("cuda", 0))
    res = 1024 if sys.argv[1] == "sdxl" else 512
    for _ in range(2):
        p(prompt="a fox", num_inference_steps=10, height=res, width=res)
    torch.cuda.synchronize()
    del p
net = load_esrgan("xinntao/RealESRGAN_x4plus", "cuda:0")
img = Image.fromarray((np.random.default_rng(0).random((512, 512, 3)) * 255).astype(np.uint8))
for _ in range(3): upscale_x4(net, img)
torch.cuda.synchronize()
T = {k: [] for k in ("convert", "h2d", "graph", "d2h", "fromarray", "total", "pinned_d2h", "upscale_x4")}
pin = torch.empty((2048, 2048, 3), dtype=torch.uint8, pin_memory=True)
for _ in range(10):
    t0 = time.perf_counter(); arr = np.asarray(img.convert("RGB")); t1 = time.perf_counter()
    x = torch.from_numpy(arr).to("cuda:0")[None]; torch.cuda.synchronize(); t2 = time.perf_counter()
    y = _run_u8(net, x); torch.cuda.synchronize(); t3 = time.perf_counter()
    h = y[0].cpu().numpy(); t4 = time.perf_counter()
    im = Image.fromarray(h); t5 = time.perf_counter()
    pin.copy_(y[0], non_blocking=True); torch.cuda.synchronize(); t6 = time.perf_counter()
    T["convert"].append(t1 - t0); T["h2d"].append(t2 - t1); T["graph"].append(t3 - t2); T["d2h"].append(t4 - t3)
    T["fromarray"].append(t5 - t4); T["total"].append(t5 - t0); T["pinned_d2h"].append(t6 - t5)
    t7 = time.perf_counter(); upscale_x4(net, img); torch.cuda.synchronize(); T["upscale_x4"].append(time.perf_counter() - t7)
print(sys.argv[1:], {k: round(1000 * statistics.median(v), 3) for k, v in T.items()},
      "allocated GB", round(torch.cuda.memory_allocated() / 1e9, 2), "reserved GB", round(torch.cuda.memory_reserved() / 1e9, 2))
