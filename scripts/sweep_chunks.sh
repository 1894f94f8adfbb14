# chunks-per-stream sweep of the fused kernel (CRLOT_CHUNKS override), one process per setting
set -e
for cfg in headline config2 config4; do
  for n in 4 8 12 15 16 20 24 32 48 64 96; do
    CRLOT_CHUNKS=$n BC_ONLY=$cfg timeout -k 10 60 python scripts/bench_configs.py 2>/dev/null | sed "s/^/n=$n /"
  done
done
