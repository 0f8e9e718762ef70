#!/bin/bash
# kernel-level A/B: the fixed probe workload (tools/pmc_probe.py: G1 MSM 2^20 x reps, NTT 2^22 x
# reps) under --kernel-trace --stats once per library variant (paths relative to the package),
# printing each variant's per-kernel averages.  tools/gpu_kab.sh lib/a.so lib/b.so ...
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for L in "$@"; do
  i=$((i+1))
  mkdir -p $R/gpurun_out/kab$i
  cd /tmp || exit 1
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kab$i \
    -o run --output-format csv -- python3 $R/tools/pmc_probe.py --reps 5 > $R/gpurun_out/kab$i/probe.txt 2>&1 || exit 1
  cd $R && echo "== $L" && python3 tools/prof_summary.py $(find gpurun_out/kab$i -name "*kernel_stats.csv") "$L" | grep -v k_gen_bases | head -24
done
