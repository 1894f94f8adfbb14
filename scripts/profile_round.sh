#!/bin/bash
# Round profile: kernel trace + stats of the bench command, then PMC traffic
# passes (FETCH_SIZE, WRITE_SIZE, SQ) each in its own rocprofv3 run.
# Usage: bash scripts/profile_round.sh rNN
set -u
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 $OUT/$name.log; exit $rc; fi
}
run trace 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 50 --no-cpu-baseline
run fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d $OUT/fetch -o run --output-format csv -- python3 scripts/prof_driver.py --reps 3
run write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d $OUT/write -o run --output-format csv -- python3 scripts/prof_driver.py --reps 3
run sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY --kernel-trace --stats -d $OUT/sq -o run --output-format csv -- python3 scripts/prof_driver.py --reps 3
run lds 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --stats -d $OUT/lds -o run --output-format csv -- python3 scripts/prof_driver.py --reps 3
run valu 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --stats -d $OUT/valu -o run --output-format csv -- python3 scripts/prof_driver.py --reps 3
echo "== done"
