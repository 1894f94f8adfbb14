set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/p15_gain.log
for nh in "960 240" "480 120"; do
  set -- $nh
  for d in 0 1; do
    echo "N=$1 H=$2 DPRE=$d" >> gpurun_out/p15_gain.log
    CRLOT_P15_DPRE=$d BG_N=$1 BG_H=$2 timeout -k 10 120 python scripts/bench_gain.py >> gpurun_out/p15_gain.log 2>&1 || exit $?
  done
done
cat gpurun_out/p15_gain.log
