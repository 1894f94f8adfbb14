# GRBM cycles, VALU / LDS instruction counts and waves: K_pair vs the half-wave walker
# (needs a library built with -DCRLOT_PAIR32_EXPERIMENT: make -C crlot-dsp_amd/csrc with pair32.o rebuilt under that flag)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/p32_pmc
mkdir -p $OUT
for cfg in base p32; do
  if [ $cfg = p32 ]; then export CRLOT_PAIR32=1 CRLOT_CHUNKS=4; else unset CRLOT_PAIR32 CRLOT_CHUNKS; fi
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-trace -d $OUT/$cfg -o run --output-format csv -- python3 scripts/prof_driver.py --reps 3 > $OUT/$cfg.log 2>&1 || { echo "$cfg rc=$?"; tail -5 $OUT/$cfg.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
for cfg in ("base", "p32"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/p32_pmc/{cfg}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "stft_ola" in r["Kernel_Name"]:
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(json.dumps({"cfg": cfg, "kernel": k[:60], **{c: sum(v) / len(v) for c, v in d.items()}}))
PY
