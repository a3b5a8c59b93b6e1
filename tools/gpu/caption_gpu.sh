#!/bin/bash
# Captioning GPU tests (GIT, BLIP-2 OPT / Flan-T5, ViT-GPT2 bf16 vs fp32).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_git_caption.py tests/test_blip2_caption.py tests/test_vit_gpt2_caption.py > gpurun_out/caption_gpu.txt 2>&1 || { tail -30 gpurun_out/caption_gpu.txt; exit 1; }
tail -6 gpurun_out/caption_gpu.txt
