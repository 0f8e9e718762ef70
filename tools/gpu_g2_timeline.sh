#!/bin/bash
# per-dispatch timeline of one G2 MSM 2^20 (config #5's inputs), tools/g2_probe.py under --kernel-trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/tlg && mkdir -p $R/gpurun_out/tlg
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tlg -o run --output-format csv -- \
  python3 $R/tools/g2_probe.py > $R/gpurun_out/tlg/probe.txt 2>&1 || exit 1
cd $R && python3 tools/timeline.py $(find gpurun_out/tlg -name "*kernel_trace.csv") 1 > gpurun_out/tlg/tl.txt && cat gpurun_out/tlg/tl.txt
