# New drop-in surfaces on the GPU: tests, then the e2e harness counterpart.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_dropin.py tests/test_ola_object.py tests/test_cpp_dropin.py > gpurun_out/dropin.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -25 gpurun_out/dropin.log
if [ $rc -eq 0 ]; then
  timeout -k 10 120 ./harness/e2e_bench 256 200 > gpurun_out/e2e_256.json && timeout -k 10 120 ./harness/e2e_bench 512 200 > gpurun_out/e2e_512.json
  echo "e2e rc=$?"
  cat gpurun_out/e2e_256.json gpurun_out/e2e_512.json
fi
