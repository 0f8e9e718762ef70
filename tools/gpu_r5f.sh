#!/bin/bash
# round 5: accumulation chunk length A/B (16 / 22 / 29) and the config #5 priority overlap
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT/midnight-bls12-381-cuda_amd/lib
for L in libbls12_381_mi355x.so var_c22.so var_c29.so libbls12_381_mi355x.so var_c22.so var_c29.so; do
  MBLS_LIB=$R/$L timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 --msm-batch 0 --msm-total-log 0 > gpurun_out/r5_chunk_$L.json 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['msm_stage_ms'])" gpurun_out/r5_chunk_$L.json $L
done
timeout -k 10 300 python bench.py --no-cpu --steps 6 --msm-batch 0 --msm-total-log 0 > gpurun_out/r5_mix.json 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r5_mix.json').read().splitlines()[-1]); m=d['mix_g2msm_batched_ntt']; print({k:m[k] for k in ('g2_msm_ms','batched_ntt_ms','overlapped_ms','sum_isolated_ms','overlap_ratio','overlapped_equal_priority_ms','overlapped_outputs_bit_identical')})"
