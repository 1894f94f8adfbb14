set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_concurrency.py tests/test_gpu_multirank.py > gpurun_out/conc.log 2>&1
rc=$?
echo "new rc=$rc"
if [ $rc -eq 0 ]; then
  CRLOT_LIB=$PWD/crlot-dsp_amd/ctl/libcrlot_dsp_oldabi.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_concurrency.py -k "flagged_chunks or host_threads" > gpurun_out/conc_oldabi.log 2>&1
  echo "oldabi rc=$?"
fi
tail -30 gpurun_out/conc.log
