#!/bin/bash
# full GPU suite + smoke() + the closing profile set and bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4f_gpu_suite.txt 2>&1 || { tail -40 gpurun_out/r4f_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r4f_gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.txt 2>&1 || { tail -20 gpurun_out/r4f_smoke.txt; exit 1; }
tail -2 gpurun_out/r4f_smoke.txt
bash tools/gpu_profiles.sh > gpurun_out/profiles.log 2>&1 || { tail -30 gpurun_out/profiles.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err || { tail -20 gpurun_out/r4f_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4f_bench.json')); print(d['value'], d['ntt_per_sec'], d['msm_step_ms']['median_ms'], d.get('bit_exact'))"
