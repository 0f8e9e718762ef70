#!/bin/bash
# run the GPU parity suite on the box (verbose per-test lines to a file so progress is visible)
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -x -v -p no:cacheprovider "$@" 2>&1 | tee gpurun_out/pytest_gpu.txt | grep -E "PASSED|FAILED|ERROR|passed|failed|error" 
exit ${PIPESTATUS[0]}
