#!/bin/bash
# round 5: accumulate-event overlap for config #5 -- test, timeline, bench mix leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_boundary.py -k "accumulate_event or multi_device_entry" -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_ev_tests.txt 2>&1 || { tail -n 30 gpurun_out/r5_ev_tests.txt; exit 1; }
tail -n 1 gpurun_out/r5_ev_tests.txt
./tools/gpu_r5g.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 6 --msm-batch 0 --msm-total-log 0 > gpurun_out/r5_mix2.json 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r5_mix2.json').read().splitlines()[-1]); m=d['mix_g2msm_batched_ntt']; print(d['value'], d['ntt_per_sec'], {k:m[k] for k in ('g2_msm_ms','batched_ntt_ms','overlapped_ms','sum_isolated_ms','overlap_ratio','overlapped_equal_priority_ms','overlapped_outputs_bit_identical')})"
