#!/bin/bash
# Stall counters of the MSM front kernels (k_digits_part, k_part_sort, k_glv_prep) and the
# tail's level kernels: two SQ passes over tools/pmc_probe.py (G1 only), summarised per kernel.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/front_pmc
rm -rf $O && mkdir -p $O
cd /tmp || exit 1
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- \
    python3 $R/tools/pmc_probe.py --reps 3 --g2-reps 0 --ntt-log 0 > $O/probe_p$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $O/probe_p$i.txt; exit 1; }
done
cd $R && python3 tools/pmc_summary.py $O > $O/summary.json && python3 - $O/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, r in d.items():
    if any(x in k for x in ("k_digits_part", "k_part_sort", "k_glv_prep", "k_reduce_scaled", "k_bucket_small", "k_final", "k_scan", "k_chunk")):
        print(k, {c: round(v, 1) for c, v in r.items()})
PY
