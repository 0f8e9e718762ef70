#!/bin/bash
# round 6: NTT pass counters (current library) + NTT variants (waves per SIMD, XCD mapping)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for V in "" v_w4 v_w3 v_xcd; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/ntt_time.py 22 50 2>/dev/null || exit 1
done > gpurun_out/r6b_variants.txt
cat gpurun_out/r6b_variants.txt
bash tools/gpu_valu_pmc.sh "" > gpurun_out/r6b_pmc.txt 2>&1 || { tail -20 gpurun_out/r6b_pmc.txt; exit 1; }
cat gpurun_out/r6b_pmc.txt
