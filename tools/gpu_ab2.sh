#!/bin/bash
# One box, several A/Bs: the -m gpu suite, then bench.py (no CPU / mix legs) under each setting of
# the argument list (environment assignments), then a kernel trace of the headline MSM loop.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab2
mkdir -p $O
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 240 python bench.py --no-cpu --no-mix --steps 10 > $O/$i.json 2> $O/$i.err || { tail -20 $O/$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ntt_per_sec'], d['msm_stage_ms'], d['msm_batch']['msm_per_sec'], d['msm_batch']['members_equal_single_msm'], 'host', d['msm_host_scalars_per_sec'], d['msm_pageable_host_per_sec'], 'vec', {k: v['gb_per_s'] for k, v in d['vecops'].items() if k != 'note'})" $O/$i.json "$E"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --headline-only --steps 5 --warmup 1 --no-cpu > $O/trace.txt 2>&1 || exit 1
cd $R && python3 tools/timeline.py $(find $O/prof -name "*kernel_trace.csv") > $O/timeline.txt 2>&1; tail -22 $O/timeline.txt
