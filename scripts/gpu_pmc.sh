#!/bin/bash
# PMC passes (each its own rocprofv3 run, --kernel-trace/--stats only beside --pmc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="${PMC_ARGS:-}"
i=0
run_pass() {
  i=$((i+1))
  echo "== pass $i: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python3 scripts/prof_driver.py $ARGS > $OUT/p$i.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 3 $OUT/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run_pass SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
run_pass SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT
[ -z "${SKIP_TRAFFIC:-}" ] && run_pass FETCH_SIZE
[ -z "${SKIP_TRAFFIC:-}" ] && run_pass WRITE_SIZE
run_pass SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32
echo "== pmc done"
