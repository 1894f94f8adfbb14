#!/bin/bash
# Parity tests against the newest variant (CRLOT_LIB), then interleaved A/Bs of
# abtmp/*.so at the headline, config 3 (4096/1024) and config 4 batched (512/128),
# and GRBM/VALU counters per library at the headline.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
NEW=${NEW:-abtmp/libcrlot_dsp_pk2v.so}
CRLOT_LIB=$PWD/$NEW timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walker_routing.py tests/test_gpu_concurrency.py -m gpu -x -q -p no:cacheprovider -k "pair or frame or golden or burst or seam or walker or conc or interleaved or gain" --timeout 120 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4d_tests.log; [ $rc -eq 0 ] || exit $rc
for shape in 1024/256 4096/1024 512/128; do
  n=${shape%/*}; h=${shape#*/}
  AB_N=$n AB_H=$h AB_ROUNDS=10 AB_GLOB="abtmp/*.so" timeout -k 10 400 python scripts/ab_bench.py > gpurun_out/ab_r4d_$n.log 2>&1 || { tail -20 gpurun_out/ab_r4d_$n.log; exit 1; }
  echo "== $shape"; tail -3 gpurun_out/ab_r4d_$n.log
done
PMC="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
for lib in abtmp/*.so; do
  n=$(basename $lib .so)
  for shape in 1024/256 4096/1024; do
    sn=${shape%/*}; sh=${shape#*/}
    CRLOT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/r4d_cyc_${n}_$sn -o run --output-format csv -- python3 scripts/prof_driver.py --reps 12 --n $sn --h $sh > gpurun_out/r4d_cyc_${n}_$sn.log 2>&1 || { echo "$n $sn failed"; tail -3 gpurun_out/r4d_cyc_${n}_$sn.log; exit 1; }
  done
done
