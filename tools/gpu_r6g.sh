#!/bin/bash
# round 6: limb-bound tests (G1 r28, NTT r29, G2 pair r28), NTT timing, full GPU suite, bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_limbs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6g_limbs.txt 2>&1 || { tail -n 40 gpurun_out/r6g_limbs.txt; exit 1; }
tail -n 2 gpurun_out/r6g_limbs.txt
timeout -k 10 120 python -u tools/ntt_time.py 22 50 > gpurun_out/r6g_ntt.txt 2>/dev/null || exit 1
cat gpurun_out/r6g_ntt.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6g_suite.txt 2>&1 || { tail -n 40 gpurun_out/r6g_suite.txt; exit 1; }
tail -n 3 gpurun_out/r6g_suite.txt
timeout -k 10 400 python -u bench.py --no-cpu --steps 20 > gpurun_out/r6g_bench.json 2> gpurun_out/r6g_bench.err || { tail -20 gpurun_out/r6g_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r6g_bench.json'))
m=d.get('mix_g2msm_batched_ntt',{})
print(d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d.get('roofline_valu',{}).get('frac'), d.get('roofline_ntt',{}).get('valu_frac'))
print('g2', m.get('g2_msm_ms'), m.get('g2_accumulate_ms'), m.get('overlapped_ms'), m.get('overlapped_outputs_bit_identical'))"
