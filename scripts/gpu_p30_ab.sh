# K_pair30 launch variants (CRLOT_P30_VARIANT 0 / 1 / 2), interleaved, at N = 1920
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pair30 or pairn" > gpurun_out/p30_tests.log 2>&1 || { tail -30 gpurun_out/p30_tests.log; exit 1; }
tail -1 gpurun_out/p30_tests.log
: > gpurun_out/p30_ab.jsonl
for r in 1 2; do
  for v in 0 1 2; do
    CRLOT_P30_VARIANT=$v P15_SHAPES=1920/480,1920/960,1920/240 timeout -k 10 200 python -u scripts/p15_hops.py 2>/dev/null | sed "s/^{/{\"variant\": $v, /" >> gpurun_out/p30_ab.jsonl || exit 1
  done
done
cat gpurun_out/p30_ab.jsonl
