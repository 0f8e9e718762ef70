#!/bin/bash
# round 6: quad-lane final inversion (shipped) vs v_fq0; NTT pricing variants on the non-persistent pass; full GPU suite
set -o pipefail
mkdir -p gpurun_out/r6j
O=gpurun_out/r6j
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.txt 2>&1 || { tail -n 30 $O/suite.txt; exit 1; }
tail -n 2 $O/suite.txt
for rep in 1 2; do
for V in "" v_fq0; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ntt_per_sec'), d.get('msm_stage_ms'))" || exit 1
done
done > $O/final_ab.txt
cat $O/final_ab.txt
for V in "" v_np_m4 v_np_e1 v_np_e2 v_np_e3 v_np_e4; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/ntt_time.py 22 50 2>/dev/null || exit 1
done > $O/ntt_variants.txt
cat $O/ntt_variants.txt
