# PMC passes on K_pairN (one rocprofv3 run per pass), PN_SHAPE as scripts/pairn_prof.py
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${PMC_TAG:-pairn}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_CYCLES SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python3 scripts/pairn_prof.py > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc_{os.environ.get('PMC_TAG', 'pairn')}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if os.environ.get("PMC_KERNEL", "k_pairn") in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:24s} {sum(v)/len(v):.5g}  (n={len(v)})")
PY
