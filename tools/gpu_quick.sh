#!/bin/bash
# Quick GPU iteration: the -m gpu suite, then A/B of library variants (tools/ab.sh arguments),
# then a kernel-trace of the ICICLE vs raw MSM paths (tools/msm_paths_probe.py).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/q
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/q/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/q/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/q/pytest_gpu.txt
bash tools/ab.sh "$@" || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/q/prof -o run --output-format csv -- \
  python3 $R/tools/msm_paths_probe.py --reps 5 > $R/gpurun_out/q/paths.txt 2>&1 || exit 1
cd $R && KS=$(find gpurun_out/q/prof -name "*kernel_stats.csv") && python3 tools/prof_summary.py $KS "paths probe" \
  > gpurun_out/q/paths_stats.md && head -24 gpurun_out/q/paths_stats.md
