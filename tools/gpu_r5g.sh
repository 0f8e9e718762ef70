#!/bin/bash
# round 5: config #5 timeline with the G2 MSM on a high-priority stream (and with equal priorities)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for M in prio equal; do
  rm -rf $R/gpurun_out/mix_$M && mkdir -p $R/gpurun_out/mix_$M
  A=""; [ $M = equal ] && A="--equal"
  cd /tmp || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/mix_$M -o run --output-format csv -- \
    python3 $R/tools/mix_probe.py $A > $R/gpurun_out/mix_$M/probe.txt 2>&1 || exit 1
  cd $R && python3 tools/mix_timeline.py $(find gpurun_out/mix_$M -name "*kernel_trace.csv") > gpurun_out/mix_$M/tl.txt || exit 1
  tail -n 3 gpurun_out/mix_$M/tl.txt
done
