#!/bin/bash
# drop-in tests, the pipeline harness (release), then A/B on the variant build:
# copy engine + two FFT launches vs zero-copy + fused launch, batch-start phases traced
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_cpp_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4_pipe_tests8.log 2>&1; rc=$?
tail -3 gpurun_out/r4_pipe_tests8.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r4_pipe_tests8.log | head -30; exit $rc; }
timeout -k 10 120 ./harness/pipeline_bench 200 > gpurun_out/pipe_diag9.log 2>&1 || exit 1
cat gpurun_out/pipe_diag9.log
for i in 1 2; do
  for cfg in "0 0" "3 1" "0 1" "3 0"; do
    set -- $cfg
    CRLOT_BATCH_TRACE=1 CRLOT_BATCH_ZC=$1 CRLOT_BATCH_FUSE=$2 timeout -k 10 120 ./abtmp/pipeline_bench_ab 200 > gpurun_out/pipe_ab_$1$2_$i.log 2>&1 || exit 1
    echo "zc=$1 fuse=$2 $(python3 -c "
import json,sys
L=open('gpurun_out/pipe_ab_$1$2_$i.log').read().splitlines()
d=json.loads([l for l in L if l.startswith('{')][0]); t=[l for l in L if l.startswith('batch_trace')]
print(d['literal']['total_us_p50'], d['interleaved']['total_us_p50'], d['interleaved']['first_forward_us_p50'], t[-1] if t else '')")"
  done
done
