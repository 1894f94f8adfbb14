# K_pairN: parity subset + throughput at the any-size shapes
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pairn or pair15 or pair30 or any_size" > gpurun_out/pn_quick_tests.log 2>&1 || { tail -30 gpurun_out/pn_quick_tests.log; exit 1; }
tail -1 gpurun_out/pn_quick_tests.log
P15_SHAPES="${SHAPES:-1764/441,882/441,1764/441,882/441,1000/250,640/320,400/160,320/160}" timeout -k 10 200 python -u scripts/p15_hops.py > gpurun_out/pn_quick.jsonl 2>/dev/null || exit 1
cat gpurun_out/pn_quick.jsonl
