# MI355X worker image (reference: Dockerfile, pytorch/pytorch CUDA base).
# Base: ROCm PyTorch; the HIP kernels are compiled for gfx950 at build time.
FROM rocm/pytorch:latest

RUN apt-get update && apt-get install -y --no-install-recommends ffmpeg && rm -rf /var/lib/apt/lists/*

WORKDIR /sdaas
COPY requirements.txt .
RUN pip install --no-cache-dir -r requirements.txt

COPY . .
ENV PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    SDAAS_ROOT=/sdaas/config \
    HF_HOME=/sdaas/models
RUN python -m chiaswarm_amd._build

# model weights (safetensors, diffusers layout) are bind-mounted:
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video \
#     -v $HOME/.cache/huggingface:/sdaas/models -e SDAAS_TOKEN=... image
VOLUME ["/sdaas/models", "/sdaas/config"]
CMD ["python", "-m", "swarm.worker"]
