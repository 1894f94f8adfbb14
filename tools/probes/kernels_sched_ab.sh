# A/B of the kernels.hip scheduler (per-frame walkers, K_pair4k/2k/512 two-regime walkers):
# put a library linked with kernels.o built under -amdgpu-sched-strategy=max-ilp in abvar/ first.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for nh in "4096 1024" "1000 250" "640 320" "2048 512" "512 128"; do set -- $nh
  echo "N=$1 H=$2" >> gpurun_out/kernels_sched_ab.log
  AB_N=$1 AB_H=$2 AB_GLOB='abvar/*.so' timeout -k 10 180 python -u scripts/ab_bench.py >> gpurun_out/kernels_sched_ab.log 2>&1 || exit $?
done
cat gpurun_out/kernels_sched_ab.log
