# A/B of the pair_any.hip scheduler: put variant libraries (make variant-style links with
# pair_any.o built under -amdgpu-sched-strategy=max-ilp / max-memory-clause) in abvar/ first.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for nh in "960 240" "480 120" "960 480" "960 240"; do set -- $nh
  echo "N=$1 H=$2" >> gpurun_out/p15_sched_ab.log
  AB_N=$1 AB_H=$2 AB_GLOB='abvar/*.so' timeout -k 10 180 python -u scripts/ab_bench.py >> gpurun_out/p15_sched_ab.log 2>&1 || exit $?
done
cat gpurun_out/p15_sched_ab.log
