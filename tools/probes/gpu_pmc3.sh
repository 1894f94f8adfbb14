#!/bin/bash
# VALU instruction classes of the headline kernel (one rocprofv3 pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc3
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_CVT --kernel-trace -d $OUT/p1 -o run --output-format csv -- python3 scripts/prof_driver.py --reps 3 > $OUT/p1.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc3/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "stft_ola" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
pairs = 1024 * 119 * 8
for k, v in sorted(agg.items()):
    print(f"{k:32s} {sum(v)/len(v):.4g}   per pair {sum(v)/len(v)/pairs:8.1f}")
PY
