#!/bin/bash
# per-dispatch kernel timeline of the fixed probe workload (3 G1 MSMs 2^20 + 3 NTTs 2^22)
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl -o run --output-format csv -- \
  python3 $R/tools/pmc_probe.py --reps 3 > $R/gpurun_out/tl/probe.txt 2>&1
