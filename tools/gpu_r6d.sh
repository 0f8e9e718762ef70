#!/bin/bash
# round 6: NTT 2^22 kernel trace (gaps between passes / transforms)
set -o pipefail
mkdir -p gpurun_out/r6d
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6d -o run --output-format csv -- python3 $R/tools/ntt_time.py 22 20) > gpurun_out/r6d/out.txt 2>&1 || { tail -20 gpurun_out/r6d/out.txt; exit 1; }
tail -2 gpurun_out/r6d/out.txt
find gpurun_out/r6d -name "*.csv" | head
