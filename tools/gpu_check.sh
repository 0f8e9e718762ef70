#!/bin/bash
# Quick GPU session: the parity suite (boundary tests first), then one bench line.  Every GPU step
# under its own timeout, chained so a failure ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_boundary.py tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider "$@" > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
