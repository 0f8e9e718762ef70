#!/bin/bash
# round 6: G1 accumulation + bucket sums in XYZZ -- limb / on-curve probes, full GPU suite, headline A/B vs Jacobian (v_jac)
set -o pipefail
mkdir -p gpurun_out/r6m
O=gpurun_out/r6m
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_limbs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/limbs.txt 2>&1 || { tail -n 30 $O/limbs.txt; exit 1; }
tail -n 2 $O/limbs.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.txt 2>&1 || { tail -n 30 $O/suite.txt; exit 1; }
tail -n 2 $O/suite.txt
for rep in 1 2; do
for V in "" v_jac; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ntt_per_sec'), d.get('msm_stage_ms'))" || exit 1
done
done > $O/xyzz_ab.txt
cat $O/xyzz_ab.txt
