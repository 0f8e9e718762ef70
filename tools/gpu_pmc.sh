#!/bin/bash
# HBM traffic counters on the box: FETCH_SIZE and WRITE_SIZE in SEPARATE rocprofv3 --pmc passes
# (they do not fit one TCC pass on gfx950; MI355X_MICROARCH.md "rocprofv3 PMC slots"), no
# tracing domains combined with --pmc.  Summaries -> gpurun_out/pmc/*.json via pmc_summary.py.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d $R/gpurun_out/pmc/$c -o run --output-format csv -- \
    python3 $R/tools/pmc_probe.py --reps 3 > $R/gpurun_out/pmc/probe_$c.txt 2>&1 || exit $?
done
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/pmc_summary.json && cat gpurun_out/pmc/pmc_summary.json
