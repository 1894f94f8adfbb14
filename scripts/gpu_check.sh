#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = rc, $2 = step
  case "$1" in
    0|1) return 0 ;;
    *) echo "FATAL rc=$1 in $2 -- stopping"; exit "$1" ;;
  esac
}
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 15 "$OUT/$name.log"
  stop_if_fatal $rc "$name"
  return $rc
}
MODE=${1:-all}
if [[ $MODE == sel ]]; then  # sel "<pytest -k expr>": selected GPU tests, then the bench
  step pytest_sel 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$2"
  step bench 600 python bench.py --no-cpu-baseline
fi
if [[ $MODE == all || $MODE == test ]]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if [[ $MODE == all || $MODE == smoke ]]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 600 python bench.py
fi
if [[ $MODE == all || $MODE == bench2 ]]; then  # the N-rank path through bench.py's own launcher
  step bench2 600 python bench.py --gpus 2 --no-cpu-baseline
fi
if [[ $MODE == all || $MODE == prof ]]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
  find $OUT/prof -name "*stats*" | head
fi
echo "== done $(date +%T)"
