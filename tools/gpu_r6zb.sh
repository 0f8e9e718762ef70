#!/bin/bash
# round 6: G2 lane levels chained on raw pair XYZZ records (shipped) vs Jacobian words between them
# (v_noraw) -- GPU suite, G2 2^20 time x3, kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zb
mkdir -p $O
cd $R || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1 || { tail -n 30 $O/gpu_suite.txt; exit 1; }
tail -n 3 $O/gpu_suite.txt
for V in "" v_noraw "" v_noraw "" v_noraw; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/g2_time.py --reps 7 2>/dev/null || exit 1
done 2>&1 | tee $O/g2_ab.txt
for V in "" v_noraw; do
  L=""; [ -n "$V" ] && L=$R/midnight-bls12-381-cuda_amd/lib/$V.so
  MBLS_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_${V:-ship} -o run --output-format csv -- python3 tools/g2_time.py --reps 5 > $O/prof_${V:-ship}.log 2>&1 || exit 1
done
