# K_pairN two-wave walk at 1764: LDS windows + power-of-two ring vs lean (CRLOT_PN_LEAN)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for l in 1 0; do
  CRLOT_PN_LEAN=$l timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pairn or pair15 or any_size" > gpurun_out/pn_lean_tests_$l.log 2>&1 || { echo "lean=$l tests failed"; tail -30 gpurun_out/pn_lean_tests_$l.log; exit 1; }
  echo "lean=$l $(tail -1 gpurun_out/pn_lean_tests_$l.log)"
done
: > gpurun_out/pn_lean.jsonl
for rep in 1 2 3; do
for l in 0 1; do
  CRLOT_PN_LEAN=$l P15_SHAPES="1764/441,1764/882" timeout -k 10 120 python -u scripts/p15_hops.py 2>/dev/null | sed "s/^/{\"lean\": $l, \"row\": /; s/\$/}/" >> gpurun_out/pn_lean.jsonl || exit 1
done
done
cat gpurun_out/pn_lean.jsonl
