set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cpp_dropin.py tests/test_gpu_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4_dropin.log 2>&1 || { tail -40 gpurun_out/r4_dropin.log; exit 1; }
tail -2 gpurun_out/r4_dropin.log
(cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r4_counters.txt 2>&1); echo "list rc=$?"
grep -i "valu\|busy\|inst_cycles" gpurun_out/r4_counters.txt | head -60
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench2.log 2>&1; tail -1 gpurun_out/r4_bench2.log | head -c 3000
