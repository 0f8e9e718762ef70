#!/bin/bash
# round 6: persistent NTT pass with register prefetch -- parity (shipped = 4 WG/CU, v_m3 = 3 WG/CU), timing vs v_nopipe
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ntt" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6i_ntt_tests.txt 2>&1 || { tail -n 30 gpurun_out/r6i_ntt_tests.txt; exit 1; }
tail -n 2 gpurun_out/r6i_ntt_tests.txt
MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/v_m3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ntt" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6i_ntt_tests_m3.txt 2>&1 || { tail -n 30 gpurun_out/r6i_ntt_tests_m3.txt; exit 1; }
tail -n 2 gpurun_out/r6i_ntt_tests_m3.txt
for rep in 1 2; do
for V in "" v_nopipe v_m3; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/ntt_time.py 22 50 2>/dev/null || exit 1
done
done > gpurun_out/r6i_variants.txt
cat gpurun_out/r6i_variants.txt
