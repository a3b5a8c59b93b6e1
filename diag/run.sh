#!/bin/bash
cd diag
hipcc --version | head -2
T=/usr/local/lib/python3.10/dist-packages/torch/lib
hipcc --offload-arch=gfx950 -O2 -fPIC -shared k.hip -o k_default.so && echo built1
hipcc --offload-arch=gfx950 -O2 -fPIC -shared -mcode-object-version=5 k.hip -o k_cov5.so && echo built2
hipcc --offload-arch=gfx950 -O2 -fPIC -shared k.hip -o k_torchrt.so -L$T -Wl,-rpath,$T && echo built3
for lib in k_default.so k_cov5.so k_torchrt.so ../chiaswarm_amd/lib/libcsk.so; do
  echo "== $lib"
  ldd $lib | grep -i hip
done
for lib in k_default.so k_cov5.so k_torchrt.so; do
  for w in notorch torch_selftest torch_launch; do
    echo "== $lib $w"; timeout -k 5 120 python run.py $w $PWD/$lib 2>&1 | tail -4; echo "rc=$?"
  done
done
