#!/bin/bash
# A/B: G2 bucket sums at 2 waves per SIMD (MBLS_BS_MINW=2, lib/var_bs2.so) against the default
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
for L in lib/libbls12_381_mi355x.so lib/var_bs2.so lib/libbls12_381_mi355x.so lib/var_bs2.so; do
  echo "== $L"
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 200 python tools/stage_probe.py --group g2 --log 20 --reps 5 2>/dev/null | tail -1 || exit 1
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 200 python tools/stage_probe.py --group g1 --log 20 --reps 5 2>/dev/null | tail -1 || exit 1
done
MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/var_bs2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "g2" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3
