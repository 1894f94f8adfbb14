# Drop-in surfaces on the GPU: tests, then the e2e harness counterpart at the
# reference's frame and at the any-size call server's 20 ms frames.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_dropin.py tests/test_ola_object.py tests/test_cpp_dropin.py > gpurun_out/dropin.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -25 gpurun_out/dropin.log
[ $rc -eq 0 ] || exit $rc
for nh in "1024 256" "1024 512" "960 480" "960 240" "882 441"; do
  set -- $nh
  timeout -k 10 120 ./harness/e2e_bench $2 200 $1 > gpurun_out/e2e_${1}_$2.json || { echo "e2e $1/$2 failed"; exit 1; }
  cat gpurun_out/e2e_${1}_$2.json
done
