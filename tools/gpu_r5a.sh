#!/bin/bash
# round 5, first GPU call: new parity tests, the GPU suite, the measured VALU ceilings, the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/valu_ceiling 24 > gpurun_out/r5_valu_ceiling.json 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -k "noncanonical or golden or plain_device_bases or multi_device" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_noncanon.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_suite1.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r5_bench1.txt 2>&1 || exit $?
MBLS_BENCH_SAME_DEVICE=1 MBLS_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --msm-total-log 21 --steps 4 --warmup 1 --no-cpu --no-mix --msm-batch 0 > gpurun_out/r5_bench_gpus2.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --gpus 1 --msm-total-log 21 --steps 4 --warmup 1 --no-cpu --no-mix --msm-batch 0 > gpurun_out/r5_bench_gpus1_t21.txt 2>&1 || exit $?
timeout -k 10 60 python bench.py --gpus 2 > gpurun_out/r5_bench_gpus2_refused.txt 2>&1; echo "refused rc=$?" >> gpurun_out/r5_bench_gpus2_refused.txt
# counters of the ceiling kernels (one pass each, bounded)
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES SQ_INSTS_SALU --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5_ceiling_pmc -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/valu_ceiling 22 > $GRAFT_REPO_ROOT/gpurun_out/r5_ceiling_pmc.txt 2>&1
echo "pmc rc=$?"
