#!/bin/bash
# round 6: second A/B repetition (shipped raw XYZZ buckets vs v_nobx, row segment 4 vs v_r2, wave
# threshold vs v_wm4k) and per-kernel stats of shipped vs v_nobx
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6x
mkdir -p $O
cd $R || exit 1
export TMPDIR=/tmp
for V in "" v_nobx v_r2 v_wm4k "" v_nobx v_r2 v_wm4k; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 200 python -u bench.py --headline-only --no-cpu --steps 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('msm_stage_ms'))" || exit 1
done 2>&1 | tee $O/ab.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_ship -o run -- python3 bench.py --headline-only --no-cpu --steps 10 > $O/prof_ship.log 2>&1 || exit 1
MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/v_nobx.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_nobx -o run -- python3 bench.py --headline-only --no-cpu --steps 10 > $O/prof_nobx.log 2>&1 || exit 1
for d in prof_ship prof_nobx; do echo "== $d"; f=$(find $O/$d -name "*kernel_stats.csv" | head -1); grep -E "reduce|bucket_small|final|accumulate" "$f" | cut -c1-60,200-; done
