#!/bin/bash
# G2 MSM 2^20 stage times per env setting: tools/sweep_g2.sh "MBLS_WAVE_MIN_G2=8192" ...
mkdir -p gpurun_out/sweep_g2
i=0
for S in "$@"; do
  i=$((i+1))
  env $S timeout -k 10 200 python tools/stage_probe.py --group g2 --log 20 --reps 5 > gpurun_out/sweep_g2/$i.json 2> gpurun_out/sweep_g2/$i.err || exit $?
  echo "$S | $(cat gpurun_out/sweep_g2/$i.json)"
done
