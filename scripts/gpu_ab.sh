#!/bin/bash
# A/B of crlot-dsp_amd/variants/*.so vs the base library: parity tests on the base, timing, cycles
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${AB_K:-pair or fused or frame or fq or golden or drop or stream}" > gpurun_out/ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/ab_bench.py > gpurun_out/ab.log 2>&1; rc=$?; cat gpurun_out/ab.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/cycles_ab.sh 2>&1 | tail -8
