#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_prepared.py tests/test_icicle_backend.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4j_tests.txt 2>&1 || { tail -40 gpurun_out/r4j_tests.txt; exit 1; }
tail -2 gpurun_out/r4j_tests.txt
timeout -k 10 300 python tools/c_sweep.py --group g1 --logs 8,10,11,12,13,14,15,16,17,20 --cs 0,8,10,11,16 || exit 1
timeout -k 10 300 python tools/c_sweep.py --group g2 --logs 8,10,12,13,14,15,16,17 --cs 0,11,13,16 || exit 1
