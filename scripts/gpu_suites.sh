# Drop-in tests, then the reference-harness counterparts (bench.py suites).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_dropin.py tests/test_ola_object.py tests/test_cpp_dropin.py tests/test_gpu_concurrency.py > gpurun_out/dropin.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/dropin.log
[ $rc -eq 0 ] || exit $rc
for s in e2e kernels pipeline; do
  timeout -k 10 300 python -u bench.py --suite $s > gpurun_out/suite_$s.json 2> gpurun_out/suite_$s.err || { echo "suite $s failed"; tail -5 gpurun_out/suite_$s.err; exit 1; }
  echo "suite $s ok"
done
