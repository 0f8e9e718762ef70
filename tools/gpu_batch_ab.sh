#!/bin/bash
# Batch-pipeline A/B on the box: the batch MSM tests, then bench.py's batch leg with the tails on
# the caller's stream (MBLS_BATCH_PIPE=0) and on the side stream (1), twice each, then a kernel
# trace of the piped batch (tools/batch_probe.py) for the timeline.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/batch
mkdir -p $O
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "batch or msm_g1_2_20 or stream" --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in 2 3 2 3; do
  MBLS_BATCH_PIPE=$v timeout -k 10 240 python bench.py --no-cpu --no-mix --steps 10 > $O/b$v.json 2> $O/b$v.err \
    || { tail -20 $O/b$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pipe', sys.argv[2], d['value'], d['msm_batch'])" $O/b$v.json $v
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/tools/batch_probe.py > $O/probe.txt 2>&1 || exit 1
cd $R && python3 tools/timeline_batch.py $(find $O/prof -name "*kernel_trace.csv") > $O/timeline.txt 2>&1; tail -5 $O/timeline.txt
