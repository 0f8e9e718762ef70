#!/bin/bash
# A/B tuning on the box: bench.py (MSM + NTT legs only) once per in-tree library variant.
#   tools/ab.sh lib/libbls12_381_mi355x.so lib/var_x.so ...   (paths relative to the package)
mkdir -p gpurun_out/ab
R=$GRAFT_REPO_ROOT
for L in "$@"; do
  echo "== $L"
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 240 python bench.py --no-cpu --no-mix --steps 10 \
    > gpurun_out/ab/$(basename $L).json 2> gpurun_out/ab/$(basename $L).err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ntt_per_sec'], d['msm_stage_ms'])" gpurun_out/ab/$(basename $L).json
done
