#!/bin/bash
# K_pair4k hot walker at three vs two workgroups per CU: parity subset, then
# alternating-process timing (each process reads CRLOT_PAIR4K_HOT once).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
CRLOT_PAIR4K_HOT=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_concurrency.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "4096 or 2048 or pair or hot or chunk" > $OUT/ab4k_pytest.log 2>&1 || { tail -30 $OUT/ab4k_pytest.log; exit 1; }
tail -2 $OUT/ab4k_pytest.log
for i in 1 2 3; do
  CRLOT_PAIR4K_HOT=3 BS_TAG=hot3 timeout -k 10 120 python scripts/bench_shapes.py 4096/1024 2048/512 || exit 1
  CRLOT_PAIR4K_HOT=2 BS_TAG=hot2 timeout -k 10 120 python scripts/bench_shapes.py 4096/1024 2048/512 || exit 1
done
BC_ONLY=2048 timeout -k 10 120 python scripts/bench_configs.py
CRLOT_PAIR4K_HOT=3 BC_ONLY=2048 timeout -k 10 120 python scripts/bench_configs.py
