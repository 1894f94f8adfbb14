#!/bin/bash
# drop-in tests, then the pipeline harness's per-call breakdown
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_cpp_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4_pipe_tests6.log 2>&1; rc=$?
tail -3 gpurun_out/r4_pipe_tests6.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4_pipe_tests6.log | head -20; exit $rc; }
timeout -k 10 120 ./harness/pipeline_bench 200 > gpurun_out/pipe_diag7.log 2>&1; rc=$?; cat gpurun_out/pipe_diag7.log; exit $rc
