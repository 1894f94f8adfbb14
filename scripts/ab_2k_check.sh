set -u
mkdir -p gpurun_out
AB_GLOB='abvar/*.so' AB_N=2048 AB_H=512 timeout -k 10 200 python scripts/ab_bench.py > gpurun_out/ab2k.log 2>&1 || exit 1
for i in 1 2; do
CRLOT_PAIR4K_HOT=3 BS_TAG=hot3 timeout -k 10 100 python scripts/bench_shapes.py 2048/512 >> gpurun_out/ab2k.log 2>&1 || exit 1
BS_TAG=hot2 timeout -k 10 100 python scripts/bench_shapes.py 2048/512 >> gpurun_out/ab2k.log 2>&1 || exit 1
done
