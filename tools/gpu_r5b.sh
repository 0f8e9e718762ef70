#!/bin/bash
# round 5: radix-2^28 accumulation -- bit-exactness (microbench + G1 parity tests) and timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/fq28_bench > gpurun_out/r5_fq28_bench.json 2>&1 || exit $?
cat gpurun_out/r5_fq28_bench.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "g1 or golden or noncanonical or window or glv or skewed or adversarial or exceptional or batch or bench_msm" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_r28_tests.txt 2>&1 || { tail -n 30 gpurun_out/r5_r28_tests.txt; exit 1; }
tail -n 2 gpurun_out/r5_r28_tests.txt
timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 --msm-batch 0 > gpurun_out/r5_r28_bench.json 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r5_r28_bench.json').read().splitlines()[-1]); print(d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d['roofline_valu']['frac'])"
MBLS_LIB=$GRAFT_REPO_ROOT/midnight-bls12-381-cuda_amd/lib/var_fips.so timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 --msm-batch 0 > gpurun_out/r5_fips_bench.json 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r5_fips_bench.json').read().splitlines()[-1]); print('fips', d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d['roofline_valu']['frac'])"
timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 --msm-batch 0 > gpurun_out/r5_r28_bench2.json 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r5_r28_bench2.json').read().splitlines()[-1]); print('r28', d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d['roofline_valu']['frac'])"
