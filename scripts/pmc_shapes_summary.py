"""Summarise gpurun_out/pmcs_<tag>/ (scripts/pmc_shapes.sh) into
profiles/<tag>_pmc_shapes.json: per dominant crlot kernel, the median launch
duration from the kernel trace and the per-launch medians of every counter;
HBM bytes = (2 FETCH_SIZE + WRITE_SIZE) KiB as in make_profile_summary.py
(gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md)."""
import collections
import csv
import json
import statistics
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import src_hash  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
src = f"gpurun_out/pmcs_{tag}"
per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [per dispatch]
dur = collections.defaultdict(list)
for part in ("sq", "sq2", "fetch", "write"):
    acc = collections.defaultdict(float)  # (kernel, dispatch, counter) -> sum over agents/dims
    try:
        rows = list(csv.DictReader(open(f"{src}/{part}/run_counter_collection.csv")))
    except FileNotFoundError:
        continue
    for r in rows:
        if "crlot" not in r["Kernel_Name"]:
            continue
        acc[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in acc.items():
        per[k][c].append(v)
    if part == "sq":
        for r in csv.DictReader(open(f"{src}/{part}/run_kernel_trace.csv")):
            if "crlot" in r["Kernel_Name"]:
                dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))

out = {"tag": tag, "src_hash": src_hash(), "source": "scripts/pmc_shapes.sh (rocprofv3 --pmc, one group per run) over scripts/bench_shapes.py "
       "at 1024 streams x 480000; medians per launch", "kernels": {}}
for k, cs in per.items():
    d = {c: statistics.median(v) for c, v in cs.items()}
    e = {"launches_traced": len(dur.get(k, [])),
         "median_duration_us": round(statistics.median(dur[k]) / 1e3, 1) if dur.get(k) else None,
         "counters": {c: round(v, 1) for c, v in sorted(d.items())}}
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        e["hbm_bytes_per_launch"] = round((2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024)
    if "SQ_ACTIVE_INST_VALU" in d and "GRBM_GUI_ACTIVE" in d and d["GRBM_GUI_ACTIVE"] > 0:
        # VALU-busy fraction per SIMD: active VALU cycles summed over the waves' SIMDs
        # / (GRBM cycles x 1024 SIMDs / 8 XCDs' GRBM instances counted once each)
        e["valu_inst_per_wave"] = round(d.get("SQ_INSTS_VALU", 0) / max(1.0, d.get("SQ_WAVES", 1)), 1)
    out["kernels"][k] = e
json.dump(out, open(f"profiles/{tag}_pmc_shapes.json", "w"), indent=1)
for k, e in out["kernels"].items():
    print(k[:90], e["median_duration_us"], e.get("hbm_bytes_per_launch"), e.get("valu_inst_per_wave"))
