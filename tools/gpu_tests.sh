#!/bin/bash
# run the GPU parity suite + smoke on the box (one process per step, each time-limited)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.txt
exit $rc
