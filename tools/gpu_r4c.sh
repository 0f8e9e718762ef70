#!/bin/bash
# round 4: event-marker gap microbenchmark + bench legs with precompute stage breakdowns
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gapbench2 -o gap -- ./tools/gapbench > gpurun_out/gapbench2.log 2>&1 || { tail -20 gpurun_out/gapbench2.log; exit 1; }
f=$(find gpurun_out/gapbench2 -name '*kernel_trace.csv' | head -1); python tools/gap_summary.py "$f" > gpurun_out/gapbench2_summary.txt; cat gpurun_out/gapbench2_summary.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-mix --msm-total-log 0 > gpurun_out/r4_bench3.json 2> gpurun_out/r4_bench3.err || { tail -20 gpurun_out/r4_bench3.err; exit 1; }
cat gpurun_out/r4_bench3.json
