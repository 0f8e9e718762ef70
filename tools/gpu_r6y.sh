#!/bin/bash
# round 6: lane-mode reduction levels after level 0 with 2-point segments (MBLS_SEGL_LOG=1;
# lane levels 2 / 3, lane thresholds 8192-32768 chains) vs the shipped plan, x2; kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6y
mkdir -p $O
cd $R || exit 1
export TMPDIR=/tmp
for rep in 1 2; do
for V in "" v_ll2s1 v_ll3s1 v_ll2s1m v_ll3s1w; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('msm_stage_ms'))" || exit 1
done
done 2>&1 | tee $O/ab.txt
for V in "" v_ll3s1; do
  L=""; [ -n "$V" ] && L=$R/midnight-bls12-381-cuda_amd/lib/$V.so
  MBLS_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_${V:-ship} -o run --output-format csv -- python3 bench.py --headline-only --no-cpu --no-stage-profile --steps 10 > $O/prof_${V:-ship}.log 2>&1 || exit 1
done
