#!/bin/bash
# round 6: G2 accumulation + bucket sums in pair-sliced XYZZ -- probes, GPU suite, G2 A/B vs Jacobian (v_g2jac)
set -o pipefail
mkdir -p gpurun_out/r6o
O=gpurun_out/r6o
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_limbs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/limbs.txt 2>&1 || { tail -n 30 $O/limbs.txt; exit 1; }
tail -n 2 $O/limbs.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.txt 2>&1 || { tail -n 30 $O/suite.txt; exit 1; }
tail -n 2 $O/suite.txt
for rep in 1 2; do
for V in "" v_g2jac; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/g2_time.py --reps 7 2>/dev/null || exit 1
done
done > $O/g2_ab.txt
cat $O/g2_ab.txt
