#!/bin/bash
# round 6: NTT timing (r29, one tile per workgroup), full GPU suite, bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ntt_time.py 22 50 > gpurun_out/r6f_ntt.txt 2>/dev/null || exit 1
cat gpurun_out/r6f_ntt.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6f_suite.txt 2>&1 || { tail -n 40 gpurun_out/r6f_suite.txt; exit 1; }
tail -n 3 gpurun_out/r6f_suite.txt
timeout -k 10 300 python -u bench.py --no-cpu --no-mix --steps 20 > gpurun_out/r6f_bench.json 2> gpurun_out/r6f_bench.err || { tail -20 gpurun_out/r6f_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6f_bench.json')); print(d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d.get('roofline_valu',{}).get('frac'), d.get('roofline_ntt',{}).get('valu_frac'))"
