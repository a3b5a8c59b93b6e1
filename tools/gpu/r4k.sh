#!/bin/bash
# VAE decode with the re-tuned conv tiles vs the previous table (same box), + VAE parity test.
mkdir -p gpurun_out
git_table=chiaswarm_amd/lib/tune_gfx950.json
timeout -k 10 200 python -u -m pytest tests/test_models_gpu.py -x -q -k "vae" --timeout 150 --timeout-method thread > gpurun_out/pytest_vae_r4k.log 2>&1 || { tail -30 gpurun_out/pytest_vae_r4k.log; exit 1; }
tail -1 gpurun_out/pytest_vae_r4k.log
for arm in new old new old; do
  if [ $arm = old ]; then export CSK_TUNE_FILE=profiles/tune_gfx950_before_r4k.json; else unset CSK_TUNE_FILE; fi
  timeout -k 10 200 python tools/decodeprof.py --iters 5 >> gpurun_out/decode_r4k_$arm.txt 2>&1 || exit 1
  echo "$arm: $(grep -v amdgpu gpurun_out/decode_r4k_$arm.txt | tail -1)"
done
