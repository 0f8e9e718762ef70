set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
for L in 16 24 32 43 64 86; do
  echo "== chunk $L"; MBLS_DEBUG=1 MBLS_ACC_CHUNK=$L timeout -k 10 120 python tools/stage_probe.py --log 20 --reps 5 2>&1 | grep -v "^\[mbls\]" || exit 1
done
MBLS_DEBUG=1 timeout -k 10 120 python tools/stage_probe.py --log 20 --reps 5 2>&1 | sort | uniq -c | head -5 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4/prof -o run --output-format csv -- python3 $R/tools/msm_paths_probe.py --reps 5 > $R/gpurun_out/r4/paths.txt 2>&1 || exit 1
cd $R && KS=$(find gpurun_out/r4/prof -name "*kernel_stats.csv") && python3 tools/prof_summary.py $KS "paths probe" > gpurun_out/r4/paths_stats.md && head -30 gpurun_out/r4/paths_stats.md
