#!/bin/bash
# Round-5 closing, part A: measured VALU ceilings, the full GPU suite, the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/closing
mkdir -p $O
cd $R || exit 1
timeout -k 10 120 tools/valu_ceiling 24 > $O/valu_ceiling.json 2> $O/valu_ceiling.err || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -n 30 $O/gpu_suite.txt; exit 1; }
tail -n 3 $O/gpu_suite.txt
timeout -k 10 400 python bench.py > $O/bench_line.json 2> $O/bench.err || { tail -n 20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench_line.json
