#!/bin/bash
# Round-3 closing set: the -m gpu suite, the profile set (tools/gpu_profiles.sh), a kernel trace
# of the pipelined batch MSM (tools/batch_probe.py), then the full bench line.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
bash tools/gpu_profiles.sh > $O/profiles.log 2>&1 || { tail -20 $O/profiles.log; exit 1; }
tail -12 $O/profiles.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_set/trace_batch -o run --output-format csv -- \
  python3 $R/tools/batch_probe.py > $O/prof_set/batch_probe.txt 2>&1 || exit 1
cd $R && python3 tools/timeline_batch.py $(find $O/prof_set/trace_batch -name "*kernel_trace.csv") > $O/prof_set/batch_timeline.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
