#!/bin/bash
# K_pair's paired-only walker at H = 512 / 128 (CRLOT_PAIR_HOT8 / _HOT2): parity
# tests on the base library, then interleaved A/Bs against variants/*.so.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pair or chunking or golden" > gpurun_out/hot_tests.log 2>&1; rc=$?
tail -3 gpurun_out/hot_tests.log; [ $rc -eq 0 ] || exit $rc
for h in ${AB_HOPS:-128 512}; do
  AB_H=$h timeout -k 10 300 python scripts/ab_bench.py > gpurun_out/hot_ab$h.log 2>&1; rc=$?; tail -4 gpurun_out/hot_ab$h.log; [ $rc -eq 0 ] || exit $rc
done
