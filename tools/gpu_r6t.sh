#!/bin/bash
# round 6: NTT tile loads issued together (shipped) vs the per-element load loop (v_loop)
set -o pipefail
mkdir -p gpurun_out/r6t
O=gpurun_out/r6t
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ntt" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/ntt_tests.txt 2>&1 || { tail -n 30 $O/ntt_tests.txt; exit 1; }
tail -n 2 $O/ntt_tests.txt
for rep in 1 2 3; do
for V in "" v_loop; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/ntt_time.py 22 50 2>/dev/null || exit 1
done
done > $O/ntt_variants.txt
cat $O/ntt_variants.txt
