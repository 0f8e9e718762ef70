#!/bin/bash
# library variant with a differently-compiled ntt.hip (every other object from build/):
#   tools/build_ntt_variant.sh NAME "-DMBLS_NTT_WAVES=4 ..."  -> midnight-bls12-381-cuda_amd/lib/NAME.so
set -e
cd "$(dirname "$0")/../midnight-bls12-381-cuda_amd"
mkdir -p build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $2 \
  -I../include -Icsrc -c csrc/ntt.hip -o build_var/ntt_$1.o
objs=$(ls build/*.o | grep -v '/ntt.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/$1.so $objs build_var/ntt_$1.o
echo lib/$1.so
