#!/bin/bash
# Tail tuning session: full GPU suite, one MSM timeline (kernel trace), then an env sweep of the
# reduction plan knobs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R || exit 1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
rm -rf $O/tl && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- \
    python3 $R/bench.py --headline-only --steps 4 --warmup 1 > /dev/null 2>&1 || exit 1
cd $R && python3 tools/timeline.py $(find $O/tl -name "*kernel_trace.csv") 2
bash tools/sweep.sh "MBLS_X=0" "MBLS_RED_PIPED=0" "MBLS_ROW_SEG_LOG=4" "MBLS_ROW_SEG_LOG=2" "MBLS_WAVE_MIN=256" "MBLS_SEG0_LOG=1" "MBLS_SEG0_LOG=3" "MBLS_ACC_CHUNK=24" "MBLS_X=0"
