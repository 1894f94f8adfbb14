#!/bin/bash
# A/B of abtmp/*.so on the headline, GRBM/VALU counters per library, and the pair
# parity tests run against the newest variant (CRLOT_LIB).
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
NEW=${NEW:-abtmp/libcrlot_dsp_pk2t.so}
CRLOT_LIB=$PWD/$NEW timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walker_routing.py tests/test_gpu_concurrency.py -m gpu -x -q -p no:cacheprovider -k "pair or frame or golden or burst or seam or walker or conc or interleaved or gain" --timeout 120 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4c_tests.log; [ $rc -eq 0 ] || exit $rc
AB_ROUNDS=12 AB_GLOB="abtmp/*.so" timeout -k 10 400 python scripts/ab_bench.py > gpurun_out/ab_r4c.log 2>&1 || { tail -20 gpurun_out/ab_r4c.log; exit 1; }
tail -4 gpurun_out/ab_r4c.log
PMC="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
for lib in abtmp/*.so; do
  n=$(basename $lib .so)
  CRLOT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/r4c_cyc_$n -o run --output-format csv -- python3 scripts/prof_driver.py --reps 12 > gpurun_out/r4c_cyc_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/r4c_cyc_$n.log; exit 1; }
done
