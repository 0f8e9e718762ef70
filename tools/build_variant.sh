#!/bin/bash
# library variant with one source compiled differently (every other object from build/):
#   tools/build_variant.sh NAME SOURCE "-DFLAG=..."   e.g.  tools/build_variant.sh v_g2lds msm_g2 "-DMBLS_ACC_G2_LDS=1"
#   -> midnight-bls12-381-cuda_amd/lib/NAME.so
set -e
cd "$(dirname "$0")/../midnight-bls12-381-cuda_amd"
mkdir -p build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $3 \
  -I../include -Icsrc -c csrc/$2.hip -o build_var/$2_$1.o
objs=$(ls build/*.o | grep -v "/$2.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/$1.so $objs build_var/$2_$1.o
echo lib/$1.so
