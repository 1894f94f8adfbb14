#!/bin/bash
# batched speculation of the FrameQueue pipeline loop: GPU tests, then the pipeline and e2e suites
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_cpp_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4_pipe_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4_pipe_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r4_pipe_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --suite pipeline > gpurun_out/r4_suite_pipeline.log 2>&1 || { tail -20 gpurun_out/r4_suite_pipeline.log; exit 1; }
tail -c 1500 gpurun_out/r4_suite_pipeline.log
timeout -k 10 300 python bench.py --suite e2e > gpurun_out/r4_suite_e2e2.log 2>&1 || { tail -20 gpurun_out/r4_suite_e2e2.log; exit 1; }
tail -c 600 gpurun_out/r4_suite_e2e2.log
