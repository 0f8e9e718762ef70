#!/bin/bash
# round 6: NTT phase pricing (timing-only variants, results wrong by construction)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for V in "" v_noload v_nostore v_nobar; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/ntt_time.py 22 50 2>/dev/null || exit 1
done > gpurun_out/r6c_variants.txt
cat gpurun_out/r6c_variants.txt
