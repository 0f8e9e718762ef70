#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_devices.py tests/test_gpu_parity.py tests/test_gpu_prepared.py -k "pinned or ntt or domain or slot0 or prepared or precompute" -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4e_tests.txt 2>&1 || { tail -40 gpurun_out/r4e_tests.txt; exit 1; }
tail -3 gpurun_out/r4e_tests.txt
for i in 1 2; do timeout -k 10 120 python tools/pinned_probe.py || exit 1; done
timeout -k 10 300 python -u bench.py --headline-only --no-stage-profile --steps 20 --warmup 3 > gpurun_out/r4e_bench.json 2> gpurun_out/r4e_bench.err || { tail -20 gpurun_out/r4e_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4e_bench.json')); print(d['value'], d['ntt_per_sec'], d['msm_step_ms'])"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-mix --msm-total-log 0 > gpurun_out/r4e_bench_full.json 2> gpurun_out/r4e_bench_full.err || { tail -20 gpurun_out/r4e_bench_full.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4e_bench_full.json')); print(d['value'], d['msm_precompute_tables'], d['msm_host_scalars_per_sec'], d['msm_pageable_host_per_sec'])"
