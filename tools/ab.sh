#!/bin/bash
# A/B tuning on the box: bench.py (MSM + NTT legs only) once per in-tree library variant,
# optionally with environment settings:  tools/ab.sh lib/x.so "lib/y.so MBLS_FOO=1" ...
mkdir -p gpurun_out/ab
R=$GRAFT_REPO_ROOT
i=0
for A in "$@"; do
  i=$((i+1))
  L=${A%% *}; E=""; [ "$L" != "$A" ] && E=${A#* }
  echo "== $A"
  env $E MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 240 python bench.py --no-cpu --no-mix --steps 10 \
    > gpurun_out/ab/$i.json 2> gpurun_out/ab/$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ntt_per_sec'], d['msm_stage_ms'])" gpurun_out/ab/$i.json
done
