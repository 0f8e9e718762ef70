#!/bin/bash
# Round-6 re-entry check: GPU suite + default bench line on the current tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
cd $R || exit 1
timeout -k 10 200 tools/valu_ceiling 24 > $O/valu_ceiling.json 2> $O/valu_ceiling.err || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1 || { tail -n 30 $O/gpu_suite.txt; exit 1; }
tail -n 3 $O/gpu_suite.txt
timeout -k 10 400 python bench.py > $O/bench_line.json 2> $O/bench.err || { tail -n 20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench_line.json
