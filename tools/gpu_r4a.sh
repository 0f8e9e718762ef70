#!/bin/bash
# round 4: new device/points tests first, then the whole GPU suite, then a bench line
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_devices.py tests/test_gpu_prepared.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_new_tests.txt 2>&1 || { tail -40 gpurun_out/r4_new_tests.txt; exit 1; }
tail -3 gpurun_out/r4_new_tests.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_gpu_suite.txt 2>&1 || { tail -40 gpurun_out/r4_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r4_gpu_suite.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-total > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { tail -20 gpurun_out/r4_bench.err; exit 1; }
cat gpurun_out/r4_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gapbench -o gap -- ./tools/gapbench > gpurun_out/gapbench.log 2>&1 || { tail -20 gpurun_out/gapbench.log; exit 1; }
f=$(find gpurun_out/gapbench -name '*kernel_trace.csv' | head -1); python tools/gap_summary.py "$f" > gpurun_out/gapbench_summary.txt; cat gpurun_out/gapbench_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/headline -o hl -- python bench.py --headline-only --steps 10 --warmup 2 > gpurun_out/headline.log 2>&1 || { tail -20 gpurun_out/headline.log; exit 1; }
f=$(find gpurun_out/headline -name '*kernel_trace.csv' | head -1); python tools/timeline.py "$f" > gpurun_out/headline_timeline.txt; cat gpurun_out/headline_timeline.txt
