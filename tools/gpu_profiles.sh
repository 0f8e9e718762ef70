#!/bin/bash
# Round profile set (-> gpurun_out/prof_set, copied to profiles/rNN):
#  1. rocprofv3 --kernel-trace --stats of the headline workload alone (bench.py --headline-only);
#  2. the same for the G2 MSM 2^20 alone (config #5's MSM: tools/stage_probe.py --group g2);
#  3. PMC passes, one rocprofv3 --pmc run per counter group (no tracing domains with --pmc), over
#     tools/pmc_probe.py (the bench's 2^20 G1 MSM, 2^20 G2 MSM and 2^22 NTT calls, nothing else):
#     VALU instruction mix, HBM fetch, HBM write, L2 hit/miss;
#  4. pmc_summary.py -> pmc_summary.json (per-kernel averages per dispatch, G1 / G2 apart).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_set
rm -rf $O && mkdir -p $O/pmc
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 $R/bench.py --headline-only --no-stage-profile --steps 10 --warmup 2 > $O/headline_bench.json 2> $O/headline_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_g2 -o run --output-format csv -- \
  python3 $R/tools/stage_probe.py --group g2 --log 20 --reps 5 > $O/g2_stages.json 2> $O/g2_stages.err || exit 1
i=0
for P in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $O/pmc/p$i -o run --output-format csv -- \
    python3 $R/tools/pmc_probe.py --reps 3 > $O/pmc/probe_p$i.txt 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
cd $R || exit 1
KS=$(find $O/trace -name "*kernel_stats.csv") && python3 tools/prof_summary.py $KS \
  "headline only: bench.py --headline-only --steps 10 --warmup 2 (setup kernels k_gen_* included)" > $O/headline_kernel_stats.md
cp $KS $O/headline_kernel_stats.csv
KS2=$(find $O/trace_g2 -name "*kernel_stats.csv") && python3 tools/prof_summary.py $KS2 \
  "G2 MSM 2^20 alone: tools/stage_probe.py --group g2 --log 20 --reps 5 (+2 warmup; setup kernels included)" > $O/g2_kernel_stats.md
cp $KS2 $O/g2_kernel_stats.csv
# the last timed MSM (--no-stage-profile: no stage-profiler hipEvent markers, whose ~10 us dispatch
# delays showed as gaps in the round-3 timeline)
python3 tools/timeline.py $(find $O/trace -name "*kernel_trace.csv") 1 > $O/headline_timeline.txt
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.json || exit 1
head -30 $O/headline_kernel_stats.md
head -16 $O/g2_kernel_stats.md
python3 - $O/pmc_summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k in ("k_accumulate<G1>", "k_accumulate<G2>", "k_ntt_pass<true, false, false>", "k_ntt_pass<false, false, false>", "k_ntt_pass<false, true, false>"):
    r = d.get(k, {})
    print(k, {c: r.get(c) for c in ("dispatches", "SQ_INSTS_VALU", "SQ_INSTS_VALU_INT64", "hbm_bytes_per_launch", "TCC_HIT_sum", "TCC_MISS_sum",
                                    "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_LDS")})
PY
