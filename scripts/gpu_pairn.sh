# K_pairN / any-size: parity tests, then throughput at 1024 x 480 000 (pairing on, then off)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "pairn or pair15 or any_size" > gpurun_out/pairn_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/pairn_tests.log
[ $rc -eq 0 ] || exit $rc
P15_SHAPES="882/441,1764/441,1000/250,640/320,400/160,320/160,960/240" timeout -k 10 300 python -u scripts/p15_hops.py > gpurun_out/pairn_bench.jsonl 2>&1 || exit 1
cat gpurun_out/pairn_bench.jsonl
