#!/bin/bash
# Parity tests against the candidate library (CRLOT_LIB), then interleaved A/Bs of
# abtmp/*.so against the release library over the pair-walker shapes.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
NEW=${NEW:-abtmp/libcrlot_dsp_pk4.so}
CRLOT_LIB=$PWD/$NEW timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walker_routing.py tests/test_gpu_concurrency.py -m gpu -x -q -p no:cacheprovider -k "pair or frame or golden or burst or seam or walker or conc or interleaved or gain or any" --timeout 120 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4e_tests.log; [ $rc -eq 0 ] || exit $rc
for shape in ${SHAPES:-1024/256 4096/1024 960/240 480/120 1920/480}; do
  n=${shape%/*}; h=${shape#*/}
  AB_N=$n AB_H=$h AB_ROUNDS=8 AB_GLOB="abtmp/*.so" timeout -k 10 400 python scripts/ab_bench.py > gpurun_out/ab_r4e_${n}_$h.log 2>&1 || { tail -20 gpurun_out/ab_r4e_${n}_$h.log; exit 1; }
  echo "== $shape"; tail -3 gpurun_out/ab_r4e_${n}_$h.log
done
