#!/bin/bash
# interleaved A/B of the libraries AB_GLOB names against the release library (headline workload)
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
AB_ROUNDS=${AB_ROUNDS:-12} timeout -k 10 400 python scripts/ab_bench.py > gpurun_out/ab_quick.log 2>&1; rc=$?
tail -12 gpurun_out/ab_quick.log; exit $rc
