#!/bin/bash
# End-of-round GPU pass: full GPU tests, smoke, round profile (trace + PMC),
# the profile summary on the box (so the bench line's traffic is non-stale),
# the bench line, and the per-config numbers.  Each step is time-limited; the
# script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/final_$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 4 "$OUT/final_$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
rm -rf $OUT/prof_$TAG
step profile 900 bash scripts/profile_round.sh $TAG
step summary 120 python scripts/make_profile_summary.py $TAG
step bench 600 python bench.py
step configs 600 python scripts/bench_configs.py
echo "== done $(date +%T)"
