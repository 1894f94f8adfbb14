#!/bin/bash
# Kernel cycles (GRBM_GUI_ACTIVE per XCD) and clock for the base library and every
# variants/*.so on the headline workload: compares builds independent of the
# power-managed clock.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for lib in crlot-dsp_amd/libcrlot_dsp.so crlot-dsp_amd/variants/*.so; do
  n=$(basename $lib .so)
  CRLOT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/cyc_$n -o run --output-format csv -- python3 scripts/prof_driver.py --reps 12 > gpurun_out/cyc_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/cyc_$n.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/cyc_*/")):
    cc = glob.glob(d + "run_counter_collection.csv"); kt = glob.glob(d + "run_kernel_trace.csv")
    if not cc or not kt: continue
    tr = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(kt[0]))}
    g = {r["Dispatch_Id"]: float(r["Counter_Value"]) / 8 for r in csv.DictReader(open(cc[0])) if "stft_ola" in r["Kernel_Name"] and "_fix" not in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"}
    ids = sorted(g, key=int)[4:]
    cyc = sum(g[i] for i in ids) / len(ids); us = sum(tr[i] for i in ids) / len(ids) / 1e3
    print(f"{os.path.basename(d[:-1])[4:]:24s} cycles {cyc/1e6:6.3f}M  kernel {us:7.1f} us  clock {cyc/us/1e3:5.3f} GHz")
PY
