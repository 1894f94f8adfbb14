# Host-buffer streaming: resident and launch-mode tests, then the streaming suite.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py -k "stream" tests/test_gpu_concurrency.py > gpurun_out/stream_tests.log 2>&1; rc=$?
tail -3 gpurun_out/stream_tests.log; exit $rc
