#!/bin/bash
# A/B: G2 reduction plan variants (tree levels up to 2048 segments; wave layout from 4096)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
for L in lib/libbls12_381_mi355x.so lib/var_tree2k.so lib/var_wmin4k.so lib/libbls12_381_mi355x.so lib/var_tree2k.so lib/var_wmin4k.so; do
  echo "== $L"
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 200 python tools/stage_probe.py --group g2 --log 20 --reps 5 2>/dev/null | tail -1 || exit 1
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 200 python tools/stage_probe.py --group g1 --log 20 --reps 5 2>/dev/null | tail -1 || exit 1
done
