set -e
for c in 64 128 256 512; do CRLOT_WG_CHUNK=$c BC_ONLY=config3 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | sed "s/^/chunk=$c /"; done
CRLOT_WG_2048=1 BC_ONLY=2048 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | sed "s/^/wg2048 /"
BC_ONLY=2048 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | sed "s/^/wave2048 /"
