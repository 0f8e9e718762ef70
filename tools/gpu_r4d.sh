#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gapbench3 -o gap -- ./tools/gapbench > gpurun_out/gapbench3.log 2>&1 || { tail -20 gpurun_out/gapbench3.log; exit 1; }
f=$(find gpurun_out/gapbench3 -name '*kernel_trace.csv' | head -1); python tools/gap_summary.py "$f" > gpurun_out/gapbench3_summary.txt; head -12 gpurun_out/gapbench3_summary.txt
for L in lib/libbls12_381_mi355x.so lib/var_nopinkernel.so lib/libbls12_381_mi355x.so lib/var_nopinkernel.so; do
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 120 python tools/pinned_probe.py || exit 1
done
