#!/bin/bash
# Round-3 checkpoint: parity suite, a short plan A/B, the profile set, then the full bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R || exit 1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
bash tools/sweep.sh "MBLS_X=0" "MBLS_SEG0_LOG=3" "MBLS_X=0" "MBLS_SEG0_LOG=3" || exit 1
bash tools/gpu_profiles.sh || exit 1
cd $R && timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
