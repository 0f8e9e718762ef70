#!/bin/bash
# round 6: accumulation waves per SIMD (shipped 3 vs v_w2 / v_w2np at 2) and reduction-plan macros
# (level-0 segment, row segment, lane levels, wave-mode threshold) on the G1 headline
set -o pipefail
mkdir -p gpurun_out/r6v
O=gpurun_out/r6v
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
for V in "" v_w2 v_w2np v_s03 v_r2 v_r4 v_ll2 v_wm1k v_wm4k; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('msm_stage_ms'))" || exit 1
done
done 2>&1 | tee $O/ab.txt
