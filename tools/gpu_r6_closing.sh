#!/bin/bash
# Round-6 closing: measured VALU ceilings, the full GPU suite, the default bench line, then the
# profile set (kernel traces + PMC passes incl. the stall pass, tools/gpu_profiles.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/closing
mkdir -p $O
cd $R || exit 1
timeout -k 10 200 tools/valu_ceiling 24 > $O/valu_ceiling.json 2> $O/valu_ceiling.err || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1 || { tail -n 30 $O/gpu_suite.txt; exit 1; }
tail -n 3 $O/gpu_suite.txt
timeout -k 10 500 python bench.py > $O/bench_line.json 2> $O/bench.err || { tail -n 20 $O/bench.err; exit 1; }
tail -c 600 $O/bench_line.json
bash $R/tools/gpu_profiles.sh > $R/gpurun_out/prof_set.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_set.log; exit 1; }
tail -n 12 $R/gpurun_out/prof_set.log
