#!/bin/bash
# round 5: parked radix-2^28 accumulation A/B against the 2-wave and FIPS variants + G1 parity
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT/midnight-bls12-381-cuda_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "g1 or golden or noncanonical or glv or skewed or adversarial or exceptional or bench_msm" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_park_tests.txt 2>&1 || { tail -n 30 gpurun_out/r5_park_tests.txt; exit 1; }
tail -n 1 gpurun_out/r5_park_tests.txt
for L in libbls12_381_mi355x.so var_r28w2.so var_fips.so libbls12_381_mi355x.so var_r28w2.so var_fips.so; do
  MBLS_LIB=$R/$L timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 --msm-batch 0 --msm-total-log 0 > gpurun_out/r5_ab2_$L.json 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['msm_stage_ms']['msm.accumulate'], d['msm_stage_ms']['msm.total'])" gpurun_out/r5_ab2_$L.json $L
done
