#!/bin/bash
# round 4 measurement set: H2D staging microbenchmark, the profile set (trace, G2, PMC), a bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/h2dbench > gpurun_out/h2dbench.txt 2>&1 || { cat gpurun_out/h2dbench.txt; exit 1; }
cat gpurun_out/h2dbench.txt
bash tools/gpu_profiles.sh > gpurun_out/profiles.log 2>&1 || { tail -30 gpurun_out/profiles.log; exit 1; }
tail -40 gpurun_out/profiles.log
cd $R && timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r4_bench2.json 2> gpurun_out/r4_bench2.err || { tail -20 gpurun_out/r4_bench2.err; exit 1; }
cat gpurun_out/r4_bench2.json
