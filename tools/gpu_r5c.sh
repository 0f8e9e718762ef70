#!/bin/bash
# round 5: radix-2^28 accumulation A/B (3 waves / 2 waves / FIPS) + counters of the two kernels
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/fq28_bench > gpurun_out/r5_fq28_bench2.json 2>&1 || exit $?
cat gpurun_out/r5_fq28_bench2.json
R=$GRAFT_REPO_ROOT/midnight-bls12-381-cuda_amd/lib
for L in libbls12_381_mi355x.so var_r28w2.so var_fips.so libbls12_381_mi355x.so var_r28w2.so var_fips.so; do
  MBLS_LIB=$R/$L timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 --msm-batch 0 --msm-total-log 0 > gpurun_out/r5_ab_$L.json 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['msm_stage_ms']['msm.accumulate'], d['msm_stage_ms']['msm.total'])" gpurun_out/r5_ab_$L.json $L
done
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5_acc_pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --headline-only --no-cpu --steps 3 --warmup 1 --no-stage-profile > $GRAFT_REPO_ROOT/gpurun_out/r5_acc_pmc.txt 2>&1
echo "pmc rc=$?"
