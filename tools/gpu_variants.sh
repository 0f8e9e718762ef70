#!/bin/bash
# Variant libraries (paths relative to the package): the parity tests matching -k $K against each,
# then bench.py (MSM + NTT legs) once per variant, base and variants alternated twice.
#   K=ntt tools/gpu_variants.sh lib/a.so lib/b.so
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
for L in "$@"; do
  MBLS_LIB=$R/midnight-bls12-381-cuda_amd/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider -k "${K:-ntt}" > gpurun_out/pytest_$(basename $L .so).txt 2>&1 \
    || { echo "FAIL $L"; tail -20 gpurun_out/pytest_$(basename $L .so).txt; exit 1; }
  echo "parity ok $L: $(tail -1 gpurun_out/pytest_$(basename $L .so).txt)"
done
ARGS=""
for L in "$@"; do ARGS="$ARGS lib/libbls12_381_mi355x.so $L"; done
bash tools/ab.sh $ARGS $ARGS
