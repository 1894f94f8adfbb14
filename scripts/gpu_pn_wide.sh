# K_pairN one vs two waves per transform (CRLOT_PN_WIDE) at 882/441 and 1764/441
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for w in d 0 1; do
  if [ $w = d ]; then unset CRLOT_PN_WIDE; else export CRLOT_PN_WIDE=$w; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pairn or pair15 or any_size" > gpurun_out/pn_wide_tests_$w.log 2>&1 || { echo "wide=$w tests failed"; tail -30 gpurun_out/pn_wide_tests_$w.log; exit 1; }
  echo "wide=$w $(tail -1 gpurun_out/pn_wide_tests_$w.log)"
done
: > gpurun_out/pn_wide.jsonl
for rep in 1 2; do
for w in 0 1; do
  CRLOT_PN_WIDE=$w P15_SHAPES="882/441,1764/441" timeout -k 10 120 python -u scripts/p15_hops.py 2>/dev/null | sed "s/^/{\"wide\": $w, \"row\": /; s/\$/}/" >> gpurun_out/pn_wide.jsonl || exit 1
done
done
P15_SHAPES="1000/250,640/320,400/160,320/160" timeout -k 10 120 python -u scripts/p15_hops.py 2>/dev/null >> gpurun_out/pn_wide.jsonl || exit 1
cat gpurun_out/pn_wide.jsonl
