# The any-size call server on the GPU: drop-in tests, the call-phase probe, and
# the e2e suite (bench.py --suite e2e: 1024/256, 1024/512, 960/480, 960/240, 882/441).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_dropin.py tests/test_ola_object.py tests/test_cpp_dropin.py > gpurun_out/dropin.log 2>&1; rc=$?
tail -3 gpurun_out/dropin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./tools/ubench/cp_any > gpurun_out/cp_any.txt 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/cp_any.txt
timeout -k 10 400 python -u bench.py --suite e2e > gpurun_out/suite_e2e.json 2> gpurun_out/suite_e2e.err || { echo "suite failed"; tail -5 gpurun_out/suite_e2e.err; exit 1; }
echo "suite ok"
