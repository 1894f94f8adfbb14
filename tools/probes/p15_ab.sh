set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pair15 or any_size" > gpurun_out/p15_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p15_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for d in 0 1; do
    echo "DPRE=$d" >> gpurun_out/p15_ab.log
    CRLOT_P15_DPRE=$d BC_ONLY=any-size timeout -k 10 120 python scripts/bench_configs.py >> gpurun_out/p15_ab.log 2>&1 || exit $?
  done
done
cat gpurun_out/p15_ab.log
