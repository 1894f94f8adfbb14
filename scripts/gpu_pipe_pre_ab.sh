#!/bin/bash
# prelaunch A/B on the variant build (pipeline harness), interleaved runs
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  for pre in 1 0; do
    CRLOT_BATCH_PRE=$pre timeout -k 10 120 ./abtmp/pipeline_bench_ab 200 > gpurun_out/pipe_pre${pre}_$i.log 2>&1 || { tail -5 gpurun_out/pipe_pre${pre}_$i.log; exit 1; }
    echo "pre=$pre $(python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/pipe_pre${pre}_$i.log') if l.startswith('{')][0])
i=d['interleaved']; print(d['literal']['total_us_p50'], i['total_us_p50'], i['framequeue_us_p50'], i['ola_object_us_p50'], i['first_forward_us_p50'], i['destroy_us_p50'])")"
  done
done
