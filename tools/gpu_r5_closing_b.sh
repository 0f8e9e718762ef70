#!/bin/bash
# Round-5 closing, part B: the profile set (kernel traces + PMC passes, tools/gpu_profiles.sh) and
# the skewed-scalar probes (G1 with stages, G2).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_profiles.sh > $R/gpurun_out/prof_set.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_set.log; exit 1; }
tail -n 8 $R/gpurun_out/prof_set.log
cd $R || exit 1
timeout -k 10 200 python tools/skew_probe.py --stages > gpurun_out/prof_set/skew_probe_g1.txt 2>&1 || exit 1
timeout -k 10 200 python tools/skew_probe.py --group g2 > gpurun_out/prof_set/skew_probe_g2.txt 2>&1 || exit 1
tail -n 1 gpurun_out/prof_set/skew_probe_g2.txt
