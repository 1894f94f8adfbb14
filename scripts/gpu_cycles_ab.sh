#!/bin/bash
# GRBM cycles + VALU counters per launch (clock-independent A/B): CYC="lib:N/H ..." pairs
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
PMC="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
for item in $CYC; do
  lib=${item%%:*}; shape=${item#*:}; n=${shape%/*}; h=${shape#*/}; tag=$(basename $lib .so)_${n}_$h
  CRLOT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/cyc_$tag -o run --output-format csv -- python3 scripts/prof_driver.py --reps 12 --n $n --h $h > gpurun_out/cyc_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/cyc_$tag.log; exit 1; }
  echo "done $tag"
done
