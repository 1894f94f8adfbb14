#!/bin/bash
# Kernel trace + PMC passes (one counter group per rocprofv3 run) of the batched
# round trip at the given shapes; summarised by scripts/pmc_shapes_summary.py.
# Usage: bash scripts/pmc_shapes.sh TAG 4096/1024 960/240 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/pmcs_$TAG
mkdir -p $OUT
run() {
  local name=$1; shift
  echo "== $name"
  timeout -k 10 240 rocprofv3 "$@" --kernel-trace --stats -d $OUT/$name -o run --output-format csv -- python3 scripts/bench_shapes.py $SHAPES > $OUT/$name.log 2>&1
  local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || { tail -n 20 $OUT/$name.log; exit $rc; }
}
SHAPES="$*"
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
# stall split: parked (s_waitcnt / s_barrier) vs issue stalls, LDS bank conflicts
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo "== done"
