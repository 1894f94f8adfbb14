#!/bin/bash
# One parameterised GPU pass (replaces the one-off gpu_*.sh runners of rounds 1-4).
# Each step runs under its own time limit; the script stops at the first failure
# (a fault, abort or timeout ends the call: nothing more touches the GPU).
#   bash scripts/gpu_run.sh TAG STEP[:ARG] ...
# steps:
#   tests[:PYTEST_K]  python -m pytest tests -m gpu [-k PYTEST_K]
#   smoke             __graft_entry__.smoke()
#   ab[:N/H]          scripts/ab_bench.py at N/H (default 1024/256) over abtmp/*.so
#   abgain:N/H        the same with a spectral gain
#   bench             bench.py (driver flags: --steps 20 --warmup 5)
#   configs           scripts/bench_configs.py
#   suite:NAME        bench.py --suite NAME
#   profile           scripts/profile_round.sh TAG + make_profile_summary.py TAG
#   py:FILE           python FILE (a one-off probe under scripts/ or tools/)
# Logs: gpurun_out/TAG_<step>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 6 "$OUT/${TAG}_$name.log"
  [ $rc -eq 0 ] || exit $rc
}
for s in "$@"; do
  step=${s%%:*}; arg=""; [ "$step" != "$s" ] && arg=${s#*:}
  case $step in
    tests)
      if [ -n "$arg" ]; then
        run "tests" 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$arg"
      else
        run "tests" 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
      fi ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    ab)
      n=${arg%%/*}; h=${arg#*/}; [ -z "$arg" ] && n=1024 && h=256
      AB_N=$n AB_H=$h AB_GLOB="abtmp/*.so" AB_ROUNDS=${AB_ROUNDS:-8} run "ab_${n}_${h}" 400 python -u scripts/ab_bench.py ;;
    abgain)
      n=${arg%%/*}; h=${arg#*/}
      AB_GAIN=1 AB_N=$n AB_H=$h AB_GLOB="abtmp/*.so" AB_ROUNDS=${AB_ROUNDS:-8} run "abgain_${n}_${h}" 400 python -u scripts/ab_bench.py ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    configs) run configs 600 python scripts/bench_configs.py ;;
    suite) run "suite_$arg" 600 python bench.py --suite "$arg" ;;
    profile)
      rm -rf "$OUT/prof_$TAG"
      run profile 900 bash scripts/profile_round.sh "$TAG"
      run summary 120 python scripts/make_profile_summary.py "$TAG" ;;
    py) run "py_$(basename "$arg" .py)" 600 python -u "$arg" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
