#!/bin/bash
# Quick GPU pass on a freshly rebuilt tree: GPU tests, smoke, the bench line.
# Each step is time-limited; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/verify_$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 4 "$OUT/verify_$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
echo "== done $(date +%T)"
