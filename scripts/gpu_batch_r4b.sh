#!/bin/bash
# Round-4 batch: (1) interleaved A/B of abtmp/*.so on the headline, (2) GRBM cycles and
# VALU counters per library (clock-independent), (3) GPU parity of the packed-screen
# variant, (4) config-3 counters of the 4k hot walker vs the 3-wave experiment.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
AB_ROUNDS=12 AB_GLOB="abtmp/*.so" timeout -k 10 400 python scripts/ab_bench.py > gpurun_out/ab_r4b.log 2>&1 || { tail -20 gpurun_out/ab_r4b.log; exit 1; }
tail -4 gpurun_out/ab_r4b.log
PMC="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
for lib in crlot-dsp_amd/libcrlot_dsp.so abtmp/*.so; do
  n=$(basename $lib .so)
  CRLOT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/r4b_cyc_$n -o run --output-format csv -- python3 scripts/prof_driver.py --reps 12 > gpurun_out/r4b_cyc_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/r4b_cyc_$n.log; exit 1; }
done
for mode in 2 3; do
  CRLOT_LIB=$PWD/abexp/libcrlot_dsp_experiments.so CRLOT_PAIR4K_HOT=$mode timeout -k 10 120 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/r4b_4k_hot$mode -o run --output-format csv -- python3 scripts/prof_driver.py --reps 8 --n 4096 --h 1024 > gpurun_out/r4b_4k_hot$mode.log 2>&1 || { echo "4k $mode failed"; tail -3 gpurun_out/r4b_4k_hot$mode.log; exit 1; }
done
CRLOT_LIB=$PWD/abtmp/libcrlot_dsp_pk2r.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walker_routing.py tests/test_gpu_concurrency.py -m gpu -x -q -p no:cacheprovider -k "pair or frame or golden or burst or seam or walker or conc" --timeout 120 --timeout-method thread > gpurun_out/r4b_pk2r_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4b_pk2r_tests.log; exit $rc
