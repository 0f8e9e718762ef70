set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "msm" > gpurun_out/pytest_msm.txt 2>&1 || { tail -30 gpurun_out/pytest_msm.txt; exit 1; }
tail -2 gpurun_out/pytest_msm.txt
bash tools/ab.sh lib/libbls12_381_mi355x.so lib/acc_vgpr.so lib/libbls12_381_mi355x.so lib/acc_vgpr.so "lib/libbls12_381_mi355x.so MBLS_DIAG_SKIP_HEAVY=1" || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl -o run --output-format csv -- python3 $R/bench.py --headline-only --steps 4 --warmup 1 > /dev/null 2>&1 || exit 1
cd $R && python3 tools/timeline.py $(find gpurun_out/tl -name "*kernel_trace.csv") 2
