#!/bin/bash
# Env-var tuning sweep on the box: one short MSM bench per setting, e.g.
#   tools/sweep.sh "MBLS_WSEG_LOG=2" "MBLS_WSEG_LOG=3 MBLS_ROW_SEG_LOG=3"
mkdir -p gpurun_out/sweep
i=0
for S in "$@"; do
  i=$((i+1))
  env $S timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 > gpurun_out/sweep/$i.json 2> gpurun_out/sweep/$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['msm_stage_ms']; print(sys.argv[2], '|', d['value'], '| dig', s['msm.digits'], 'sort', s['msm.sort'], 'acc', s['msm.accumulate'], 'red', s['msm.reduce'], 'fin', s['msm.final'], 'bs', s['msm.bucket_sum'])" gpurun_out/sweep/$i.json "$S"
done
