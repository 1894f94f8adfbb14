#!/bin/bash
# K_pairN at 1764 by decimation in time: parity tests against the variant (CRLOT_LIB),
# then interleaved A/Bs against the release library
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
CRLOT_LIB=$PWD/abtmp/libcrlot_dsp_dit.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walker_routing.py tests/test_gpu_concurrency.py -m gpu -x -q -p no:cacheprovider -k "1764 or pairn or any_size or seam" --timeout 120 --timeout-method thread > gpurun_out/dit_tests.log 2>&1; rc=$?
tail -3 gpurun_out/dit_tests.log; [ $rc -eq 0 ] || exit $rc
for shape in 1764/441 1764/882 882/441; do
  n=${shape%/*}; h=${shape#*/}
  AB_N=$n AB_H=$h AB_ROUNDS=8 AB_GLOB="abtmp/*.so" timeout -k 10 400 python scripts/ab_bench.py > gpurun_out/ab_dit_${n}_$h.log 2>&1 || { tail -20 gpurun_out/ab_dit_${n}_$h.log; exit 1; }
  echo "== $shape"; tail -2 gpurun_out/ab_dit_${n}_$h.log
done
