#!/bin/bash
# round 6: level 0 loading bucket t - 1 while adding bucket t (shipped) vs loading after (v_nopf1 G1,
# v_nopf2 G2) and G2 lane levels after level 0 (v_g2ll*) -- GPU suite, G1 headline stages and G2 2^20 time, x2, then kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6za
mkdir -p $O
cd $R || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1 || { tail -n 30 $O/gpu_suite.txt; exit 1; }
tail -n 3 $O/gpu_suite.txt
for V in "" v_nopf1 "" v_nopf1; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('msm_stage_ms'))" || exit 1
done 2>&1 | tee $O/g1_ab.txt
for V in "" v_nopf2 v_g2ll2 v_g2ll3 v_g2ll2s2 "" v_nopf2 v_g2ll2 v_g2ll3 v_g2ll2s2; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/g2_time.py --reps 7 2>/dev/null || exit 1
done 2>&1 | tee $O/g2_ab.txt
for V in "" v_nopf1; do
  L=""; [ -n "$V" ] && L=$R/midnight-bls12-381-cuda_amd/lib/$V.so
  MBLS_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_${V:-ship} -o run --output-format csv -- python3 bench.py --headline-only --no-cpu --no-stage-profile --steps 10 > $O/prof_${V:-ship}.log 2>&1 || exit 1
done
MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/v_nopf2.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_nopf2 -o run --output-format csv -- python3 tools/g2_time.py --reps 5 > $O/prof_nopf2.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_ship2 -o run --output-format csv -- python3 tools/g2_time.py --reps 5 > $O/prof_ship2.log 2>&1 || exit 1
