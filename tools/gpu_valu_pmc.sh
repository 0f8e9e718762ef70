#!/bin/bash
# VALU / cache counter passes (one rocprofv3 --pmc pass per counter group, no tracing domains)
# over tools/pmc_probe.py (bench headline MSM + NTT 2^22), per env setting given as arguments:
#   tools/gpu_valu_pmc.sh "" "MBLS_ACC_CHUNK=16"       -> gpurun_out/valu/<i>/...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
i=0
for S in "$@"; do
  i=$((i+1))
  O=$R/gpurun_out/valu/$i
  mkdir -p $O
  k=0
  for P in "$P1" "$P2"; do
    k=$((k+1))
    (cd /tmp && env $S timeout -s KILL 90 rocprofv3 --pmc $P -d $O/p$k -o run --output-format csv -- \
      python3 $R/tools/pmc_probe.py --reps 3 > $O/probe_p$k.txt 2>&1) || { tail -5 $O/probe_p$k.txt; exit 1; }
  done
  python3 $R/tools/pmc_table.py "$S" $O/p1 $O/p2 > $O/table.json || exit 1
  echo "== [$S]"; python3 - $O/table.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, r in d.items():
    if any(x in k for x in ("k_accumulate", "k_ntt_pass", "k_bucket_small", "k_reduce_level")):
        print(k, {c: (round(v, 4) if isinstance(v, float) else v) for c, v in r.items()})
PY
done
