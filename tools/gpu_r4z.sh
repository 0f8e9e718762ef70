#!/bin/bash
# round-4 closing set: full GPU suite + smoke() + profiles + bench line (gpu_r4f.sh), then the
# skewed-scalar probe for both groups
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
bash tools/gpu_r4f.sh || exit 1
timeout -k 10 300 python tools/skew_probe.py --log 20 --reps 10 > gpurun_out/skew_g1.txt || exit 1
timeout -k 10 300 python tools/skew_probe.py --log 20 --reps 5 --group g2 > gpurun_out/skew_g2.txt || exit 1
tail -1 gpurun_out/skew_g1.txt
tail -1 gpurun_out/skew_g2.txt
