#!/bin/bash
# round 5: where the NTT pass time goes -- diagnostic variants (no twiddle loads / no barriers,
# results wrong) and SQ counters of the three 2^22 passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/midnight-bls12-381-cuda_amd/lib
for L in libbls12_381_mi355x.so var_ntt_e1.so var_ntt_e2.so libbls12_381_mi355x.so var_ntt_e1.so var_ntt_e2.so; do
  MBLS_LIB=$R/$L timeout -k 10 200 python bench.py --headline-only --no-cpu --steps 20 > gpurun_out/r5_ntt_$L.json 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['ntt_per_sec'], d['ntt_ms'], d['roofline_ntt']['pass_ms'])" gpurun_out/r5_ntt_$L.json $L
done
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5_ntt_pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --headline-only --no-cpu --steps 3 --warmup 1 --no-stage-profile > $GRAFT_REPO_ROOT/gpurun_out/r5_ntt_pmc.txt 2>&1
echo "pmc rc=$?"
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_prepared.py -k "g1 or golden or noncanonical or glv or skewed or adversarial or exceptional or bench_msm or prepared" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_bs_tests.txt 2>&1 || { tail -n 30 gpurun_out/r5_bs_tests.txt; exit 1; }
tail -n 1 gpurun_out/r5_bs_tests.txt
for L in libbls12_381_mi355x.so var_r28w2.so libbls12_381_mi355x.so var_r28w2.so; do
  MBLS_LIB=$R/$L timeout -k 10 200 python bench.py --no-cpu --no-mix --steps 10 --msm-batch 0 --msm-total-log 0 > gpurun_out/r5_bs_$L.json 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['msm_stage_ms'])" gpurun_out/r5_bs_$L.json $L
done
