#!/bin/bash
# every GPU test, smoke, then the pipeline and e2e suites (drop-in per-call numbers)
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4_all_tests4.log 2>&1; rc=$?
tail -3 gpurun_out/r4_all_tests4.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r4_all_tests4.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -5 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
timeout -k 10 300 python bench.py --suite pipeline > gpurun_out/r4_suite_pipeline5.log 2>&1 || { tail -20 gpurun_out/r4_suite_pipeline5.log; exit 1; }
timeout -k 10 300 python bench.py --suite e2e > gpurun_out/r4_suite_e2e12.log 2>&1 || { tail -20 gpurun_out/r4_suite_e2e12.log; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r4_suite_pipeline5.log') if l.startswith('{')][-1])
p=d['per_frame']; print('pipeline', p['literal']['total_us_p50'], p['interleaved']['total_us_p50'], p['interleaved']['loop_parts_us_p50'], p['cpu_oracle_1thread'])
d=json.loads([l for l in open('gpurun_out/r4_suite_e2e12.log') if l.startswith('{')][-1])
for r in d['runs']: print(r['frame'], r['hop'], r['full_pipeline']['us_per_frame'], r['harness_order']['us_per_frame'], r['per_call_us_p50'], r['cpu_oracle_1thread']['us_per_frame'])"
timeout -k 10 120 ./harness/pipeline_bench 200 > gpurun_out/pipe_diag17.log 2>&1 && cat gpurun_out/pipe_diag17.log
