# K_pairN radix-list A/B at 882/441 and 1764/441 (library built with -DCRLOT_PN_VARIANTS)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in 1 2 3; do
  CRLOT_PN_PLAN=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pairn and (882 or 1764)" > gpurun_out/pn_plan_tests_$v.log 2>&1 || { echo "plan $v tests failed"; tail -20 gpurun_out/pn_plan_tests_$v.log; exit 1; }
  tail -1 gpurun_out/pn_plan_tests_$v.log
done
: > gpurun_out/pn_plans.jsonl
for rep in 1 2; do
for v in 0 1 2 3; do
  CRLOT_PN_PLAN=$v P15_SHAPES="882/441,1764/441" timeout -k 10 120 python -u scripts/p15_hops.py 2>/dev/null | sed "s/^/{\"plan\": $v, \"row\": /; s/\$/}/" >> gpurun_out/pn_plans.jsonl || exit 1
done
done
cat gpurun_out/pn_plans.jsonl
