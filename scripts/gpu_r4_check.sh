set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_walker_routing.py tests/test_gpu_dropin.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "route or record or chunk or regimes or seam or idle or grows or chained" > gpurun_out/r4_focus.log 2>&1 || { tail -40 gpurun_out/r4_focus.log; exit 1; }
tail -3 gpurun_out/r4_focus.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4_all.log 2>&1 || { tail -40 gpurun_out/r4_all.log; exit 1; }
tail -3 gpurun_out/r4_all.log
timeout -k 10 300 python bench.py > gpurun_out/r4_bench.log 2>&1; tail -1 gpurun_out/r4_bench.log
