#!/bin/bash
# bench + rocprofv3 kernel-trace summary on the box
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py "$@" 2>&1 | tee gpurun_out/bench.txt || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.txt 2>&1
rc=$?
echo "rocprof rc=$rc"
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
exit $rc
