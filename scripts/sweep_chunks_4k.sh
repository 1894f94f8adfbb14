# Config 3 (4096/1024) against the chunk count per stream (CRLOT_CHUNKS), alternating
set -u
for i in 1 2; do
  for c in 0 1 2 3 4 6; do
    if [ $c = 0 ]; then BS_TAG=chooser timeout -k 10 100 python scripts/bench_shapes.py 4096/1024 || exit 1
    else CRLOT_CHUNKS=$c BS_TAG=chunks$c timeout -k 10 100 python scripts/bench_shapes.py 4096/1024 || exit 1; fi
  done
done
