#!/bin/bash
# round 6 final: smoke() and the default bench line on the final tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
cd $R || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -n 20 $O/smoke.txt; exit 1; }
tail -n 2 $O/smoke.txt
timeout -k 10 500 python bench.py > $O/bench_line.json 2> $O/bench.err || { tail -n 20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_line.json').read().strip().splitlines()[-1]); print(d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d['mix_g2msm_batched_ntt']['g2_msm_ms'])"
