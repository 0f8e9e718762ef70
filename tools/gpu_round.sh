#!/bin/bash
# One GPU session: parity suite, then the bench line, then a rocprofv3 kernel-trace summary of
# the headline workload ALONE (bench.py --headline-only: G1 MSM 2^20 + NTT 2^22 loops), then the
# counter list.  Every GPU step under its own timeout, chained with &&.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --headline-only --steps 10 --warmup 2 > $O/bench_headline_prof.json 2> $O/bench_headline_prof.err || exit 1
cd $R && KS=$(find $O/prof -name "*kernel_stats.csv") && python3 tools/prof_summary.py $KS "headline only: bench.py --headline-only --steps 10 --warmup 2" > $O/headline_kernel_stats.md; head -45 $O/headline_kernel_stats.md
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; true
