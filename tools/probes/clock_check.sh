#!/bin/bash
# Effective shader clock of the headline kernel on random vs zero input
# (GRBM_GUI_ACTIVE per XCD / kernel duration): a power-capped kernel clocks lower on high-toggle data.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for d in uniform zeros; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/clk_$d -o run --output-format csv -- python3 scripts/prof_driver.py --reps 20 --data $d > gpurun_out/clk_$d.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for d in ("uniform", "zeros"):
    rows = [r for r in csv.DictReader(open(glob.glob(f"gpurun_out/clk_{d}/run_counter_collection.csv")[0])) if "stft_ola" in r["Kernel_Name"]]
    tr = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(glob.glob(f"gpurun_out/clk_{d}/run_kernel_trace.csv")[0]))}
    g = {}
    for r in rows:
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            g[r["Dispatch_Id"]] = float(r["Counter_Value"]) / 8
    ids = sorted(g)[5:]
    clk = [g[i] / tr[i] for i in ids if i in tr]
    dur = [tr[i] for i in ids if i in tr]
    print(d, "kernel us %.1f" % (sum(dur) / len(dur) / 1e3), "clock GHz %.3f" % (sum(clk) / len(clk)), "cycles %.3gM" % (sum(g[i] for i in ids) / len(ids) / 1e6))
PY
