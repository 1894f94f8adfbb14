# K_pair15 at several hops: the HEAD build (libcrlot_dsp_head.so) against the tree's build, interleaved
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pair15 or any_size" > gpurun_out/p15_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p15_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/p15_hops.log
for r in 1 2; do
  for lib in libcrlot_dsp_head.so crlot-dsp_amd/libcrlot_dsp.so; do
    echo "LIB=$lib" >> gpurun_out/p15_hops.log
    P15_SHAPES=${P15_SHAPES:-} CRLOT_LIB=$PWD/$lib timeout -k 10 120 python scripts/p15_hops.py >> gpurun_out/p15_hops.log 2>&1 || exit $?
  done
done
cat gpurun_out/p15_hops.log
