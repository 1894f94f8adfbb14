#!/bin/bash
# round-4 end: the pipeline A/B (variant build), the pipeline and e2e suites,
# then the final pass (scripts/final_round.sh: all GPU tests, smoke, profile, bench, configs)
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "0 0" "3 1" "0 1" "3 0"; do
  set -- $cfg
  CRLOT_BATCH_TRACE=1 CRLOT_BATCH_ZC=$1 CRLOT_BATCH_FUSE=$2 timeout -k 10 120 ./abtmp/pipeline_bench_ab 200 > gpurun_out/pipe_ab_$1$2.log 2>&1 || { tail -5 gpurun_out/pipe_ab_$1$2.log; exit 1; }
  echo "zc=$1 fuse=$2 $(python3 -c "
import json
L=open('gpurun_out/pipe_ab_$1$2.log').read().splitlines()
d=json.loads([l for l in L if l.startswith('{')][0]); t=[l for l in L if l.startswith('batch_trace')]
print(d['literal']['total_us_p50'], d['interleaved']['total_us_p50'], d['interleaved']['first_forward_us_p50'], t[-1] if t else '')")"
done
timeout -k 10 300 python bench.py --suite pipeline > gpurun_out/r4_suite_pipeline.log 2>&1 || { tail -20 gpurun_out/r4_suite_pipeline.log; exit 1; }
tail -c 1200 gpurun_out/r4_suite_pipeline.log
timeout -k 10 300 python bench.py --suite e2e > gpurun_out/r4_suite_e2e3.log 2>&1 || { tail -20 gpurun_out/r4_suite_e2e3.log; exit 1; }
bash scripts/final_round.sh r04c
