#!/bin/bash
# the pipeline harness alone (construction, loop parts, destruction)
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./harness/pipeline_bench 200 > gpurun_out/pipe_diag12.log 2>&1; rc=$?; cat gpurun_out/pipe_diag12.log; exit $rc
