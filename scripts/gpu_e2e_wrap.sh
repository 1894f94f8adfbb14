#!/bin/bash
# drop-in tests, then the e2e suite (harness order served from the batch) and the pipeline harness
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_cpp_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4_pipe_tests13.log 2>&1; rc=$?
tail -3 gpurun_out/r4_pipe_tests13.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r4_pipe_tests9.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --suite e2e > gpurun_out/r4_suite_e2e10.log 2>&1 || { tail -20 gpurun_out/r4_suite_e2e10.log; exit 1; }
python3 -c "
import json
L=[l for l in open('gpurun_out/r4_suite_e2e10.log') if l.startswith('{')]
d=json.loads(L[-1])
for r in d['runs']: print(r['frame'], r['hop'], r['full_pipeline']['us_per_frame'], r['harness_order'], r['cpu_oracle_1thread']['us_per_frame'])"
timeout -k 10 120 ./harness/pipeline_bench 200 > gpurun_out/pipe_diag15.log 2>&1 || exit 1
cat gpurun_out/pipe_diag15.log
