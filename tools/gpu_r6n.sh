#!/bin/bash
# round 6: XYZZ accumulation ceiling (valu_ceiling 24), y parked in LDS (shipped) vs in registers (v_nopark)
set -o pipefail
mkdir -p gpurun_out/r6n
O=gpurun_out/r6n
R=$GRAFT_REPO_ROOT
timeout -k 10 200 tools/valu_ceiling 24 > $O/valu_ceiling.json 2> $O/valu_ceiling.err || { cat $O/valu_ceiling.err; exit 1; }
cat $O/valu_ceiling.json
for rep in 1 2; do
for V in "" v_nopark; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ntt_per_sec'), d.get('msm_stage_ms'), d['roofline_valu'].get('frac'))" || exit 1
done
done > $O/park_ab.txt
cat $O/park_ab.txt
