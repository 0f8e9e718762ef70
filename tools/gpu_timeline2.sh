#!/bin/bash
# per-dispatch kernel timelines of the fixed probe workload (3 G1 MSMs 2^20 + 3 NTTs 2^22),
# once per environment setting given as arguments ("" = defaults), e.g. "" "MBLS_ROW_SEG_LOG=2"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for E in "$@"; do
  i=$((i+1))
  mkdir -p $R/gpurun_out/tl$i
  cd /tmp || exit 1
  env $E timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl$i -o run --output-format csv -- \
    python3 $R/tools/pmc_probe.py --reps 3 > $R/gpurun_out/tl$i/probe.txt 2>&1 || exit 1
  cd $R && echo "== [$E]" && python3 tools/timeline.py $(find gpurun_out/tl$i -name "*kernel_trace.csv") 2
done
