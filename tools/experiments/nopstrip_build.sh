#!/bin/bash
# Experiment: rebuild one HIP object with its device .s passed through nopstrip.py,
# then link a variant library ../../crlot-dsp_amd/variants/libcrlot_dsp_nopstrip.so
# from the release objects with that object replaced.
#   bash tools/experiments/nopstrip_build.sh pair1k "-mllvm -amdgpu-sched-strategy=max-ilp"
set -euo pipefail
SRC=$1; EXTRA=${2:-}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
CS=$ROOT/crlot-dsp_amd/csrc
W=$(mktemp -d /tmp/nopstrip.XXXX)
cd "$W"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize $EXTRA \
  -I$ROOT/include -I$CS -c $CS/$SRC.hip -o $SRC.o -save-temps -### 2>&1 | grep '^ "' > cmds.txt
n=$(wc -l < cmds.txt)
for i in 1 2 3; do eval "$(sed -n ${i}p cmds.txt)"; done
DS=$SRC-hip-amdgcn-amd-amdhsa-gfx950.s
cp $DS orig.s
python3 $ROOT/tools/experiments/nopstrip.py orig.s $DS
for i in $(seq 4 $n); do eval "$(sed -n ${i}p cmds.txt)"; done
mkdir -p $ROOT/crlot-dsp_amd/variants
objs=""
for o in $(cd $CS && ls *.o); do if [ "$o" = "$SRC.o" ]; then objs="$objs $W/$SRC.o"; else objs="$objs $CS/$o"; fi; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/crlot-dsp_amd/variants/libcrlot_dsp_nopstrip.so $objs
echo "built $ROOT/crlot-dsp_amd/variants/libcrlot_dsp_nopstrip.so from $W"
