#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "ntt or vec or batch_inv or sum or boundary or icicle" > gpurun_out/r4k_tests.txt 2>&1 || { tail -40 gpurun_out/r4k_tests.txt; exit 1; }
tail -2 gpurun_out/r4k_tests.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu --msm-total-log 0 > gpurun_out/r4k_bench.json 2> gpurun_out/r4k_bench.err || { tail -20 gpurun_out/r4k_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4k_bench.json')); print(d['value'], d['ntt_per_sec'], d['ntt20_roundtrip_ms'], d['vecops'], d['mix_g2msm_batched_ntt']['g2_msm_ms'], d['mix_g2msm_batched_ntt']['batched_ntt_ms'])"
