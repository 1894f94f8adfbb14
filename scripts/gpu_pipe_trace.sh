#!/bin/bash
# kernel + copy timeline of the pipeline harness (one short run)
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pipe_trace -o run -- $GRAFT_REPO_ROOT/harness/pipeline_bench 20 > $GRAFT_REPO_ROOT/gpurun_out/pipe_trace.log 2>&1; rc=$?
tail -2 $GRAFT_REPO_ROOT/gpurun_out/pipe_trace.log; find $GRAFT_REPO_ROOT/gpurun_out/pipe_trace -name "*.csv" | head; exit $rc
