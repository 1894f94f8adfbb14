set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
CRLOT_PAIR4K_HOT=3 BS_S=1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4k3 -o run -- python scripts/bench_shapes.py 4096/1024 2048/512 > gpurun_out/prof4k3.log 2>&1
