#!/bin/bash
# round 6: G1 raw XYZZ buckets + XYZZ level 0 (shipped) -- GPU suite, then an A/B against
# v_nobx (Jacobian buckets), the accumulation at 2 waves per SIMD (v_w2 / v_w2np) and the
# reduction-plan macros (level-0 segment, row segment, lane levels, wave-mode threshold)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6w
mkdir -p $O
cd $R || exit 1
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1 || { tail -n 30 $O/gpu_suite.txt; exit 1; }
  tail -n 3 $O/gpu_suite.txt
fi
for rep in $(seq 1 ${REPS:-1}); do
for V in "" v_nobx v_w2 v_w2np v_s03 v_r2 v_r4 v_ll2 v_wm1k v_wm4k; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('msm_stage_ms'))" || exit 1
done
done 2>&1 | tee -a $O/ab.txt
