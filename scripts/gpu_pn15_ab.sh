# K_pairN vs K_pair15 at 960 / 480, and 1920 plans (library built with -DCRLOT_PN_15)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CRLOT_PN_OVER15=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pair15 or any_size or pairn" > gpurun_out/pn15_tests.log 2>&1 || { tail -30 gpurun_out/pn15_tests.log; exit 1; }
echo "over15 tests: $(tail -1 gpurun_out/pn15_tests.log)"
: > gpurun_out/pn15_ab.jsonl
for rep in 1 2; do
  P15_SHAPES="960/240,960/480,480/120,1920/480" timeout -k 10 120 python -u scripts/p15_hops.py 2>/dev/null | sed 's/^/{"kern": "pair15", "row": /; s/$/}/' >> gpurun_out/pn15_ab.jsonl || exit 1
  for v in 0 1 2 3; do
    CRLOT_PN_OVER15=1 CRLOT_PN_PLAN=$v P15_SHAPES="960/240,960/480,480/120,1920/480" timeout -k 10 120 python -u scripts/p15_hops.py 2>/dev/null | sed "s/^/{\"kern\": \"pairn$v\", \"row\": /; s/\$/}/" >> gpurun_out/pn15_ab.jsonl || exit 1
  done
done
cat gpurun_out/pn15_ab.jsonl
