#!/bin/bash
# round 6: XYZZ accumulation at 3 waves per SIMD (shipped) vs 2 waves (v_w2, y parked in LDS; v_w2np, in registers)
set -o pipefail
mkdir -p gpurun_out/r6u
O=gpurun_out/r6u
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for V in "" v_w2 v_w2np; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('msm_stage_ms'))" || exit 1
done
done > $O/waves_ab.txt
cat $O/waves_ab.txt
