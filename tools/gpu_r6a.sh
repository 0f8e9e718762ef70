#!/bin/bash
# round 6: NTT radix-2^29 products -- parity, timing, ceilings
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ntt" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6a_ntt_tests.txt 2>&1 || { tail -n 30 gpurun_out/r6a_ntt_tests.txt; exit 1; }
tail -n 3 gpurun_out/r6a_ntt_tests.txt
timeout -k 10 120 python -u tools/ntt_time.py 22 50 > gpurun_out/r6a_ntt_time.json 2>&1 || { cat gpurun_out/r6a_ntt_time.json; exit 1; }
cat gpurun_out/r6a_ntt_time.json
timeout -k 10 120 python -u tools/ntt_time.py 20 50 >> gpurun_out/r6a_ntt_time.json 2>&1 || exit 1
timeout -k 10 200 ./tools/valu_ceiling 24 > gpurun_out/r6a_valu_ceiling.json 2>&1 || { cat gpurun_out/r6a_valu_ceiling.json; exit 1; }
cat gpurun_out/r6a_valu_ceiling.json
