#!/bin/bash
# round 6: limb-bound tests, full GPU suite, NTT persistent-pass timing, bench line
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_limbs.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6e_limbs.txt 2>&1 || { tail -n 40 gpurun_out/r6e_limbs.txt; exit 1; }
tail -n 3 gpurun_out/r6e_limbs.txt
for V in "" v_g5; do
  L=""; [ -n "$V" ] && L="MBLS_LIB=$R/midnight-bls12-381-cuda_amd/lib/$V.so"
  echo "== ${V:-shipped}"
  env $L timeout -k 10 120 python -u tools/ntt_time.py 22 50 2>/dev/null || exit 1
done > gpurun_out/r6e_ntt.txt
cat gpurun_out/r6e_ntt.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6e_suite.txt 2>&1 || { tail -n 40 gpurun_out/r6e_suite.txt; exit 1; }
tail -n 3 gpurun_out/r6e_suite.txt
timeout -k 10 300 python -u bench.py --no-cpu --no-mix --steps 20 > gpurun_out/r6e_bench.json 2> gpurun_out/r6e_bench.err || { tail -20 gpurun_out/r6e_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6e_bench.json')); print(d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d.get('roofline_valu',{}).get('frac'), d.get('roofline_ntt',{}).get('valu_frac'))"
