set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_cpp_dropin.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4_batch.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/r4_batch.log | tail -30; tail -60 gpurun_out/r4_batch.log; exit 1; }
tail -3 gpurun_out/r4_batch.log
timeout -k 10 300 python bench.py --suite e2e > gpurun_out/r4_e2e.log 2>&1; tail -c 3000 gpurun_out/r4_e2e.log
timeout -k 10 900 bash scripts/profile_round.sh r04a > gpurun_out/r4_prof.log 2>&1 || { tail -20 gpurun_out/r4_prof.log; exit 1; }
timeout -k 10 120 python scripts/make_profile_summary.py r04a > gpurun_out/r4_prof_summary.log 2>&1; tail -30 gpurun_out/r4_prof_summary.log
