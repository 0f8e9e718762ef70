#!/bin/bash
# round 6: G2 accumulation variants (register prefetch / LDS-DMA prefetch / 3 waves), valu ceilings
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for V in "" v_g2lds v_g2w3; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/g2_time.py --reps 7 2>/dev/null || exit 1
done > gpurun_out/r6h_g2.txt
cat gpurun_out/r6h_g2.txt
timeout -k 10 300 ./tools/valu_ceiling 24 > gpurun_out/r6h_valu_ceiling.json 2>&1 || { cat gpurun_out/r6h_valu_ceiling.json; exit 1; }
cat gpurun_out/r6h_valu_ceiling.json
