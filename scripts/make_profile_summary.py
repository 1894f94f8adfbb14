"""Turn gpurun_out/prof_<tag>/ into committed summaries under profiles/:
  profiles/<tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats of bench.py
  profiles/<tag>_kernel_stats_by_grid.csv  the same trace per (kernel, grid size)
  profiles/<tag>_pmc_summary.json    per-launch PMC values of the fused kernel and
                                     the HBM traffic figure bench.py reports.
HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE reads
half the bytes of a coalesced streaming read on gfx950 (MI355X_MICROARCH.md,
HBM section); WRITE_SIZE is exact for streaming stores.  Our reads are 8 B/lane
dwordx2; the doubled value lands at 1.05x the algorithmic read bytes, which the
recomputed warm-up frames (3 per 125-frame chunk) and the normaliser table explain."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import src_hash  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = f"gpurun_out/prof_{tag}"
os.makedirs("profiles", exist_ok=True)
stats = glob.glob(f"{src}/trace/run_kernel_stats.csv")
if stats:
    shutil.copy(stats[0], f"profiles/{tag}_kernel_stats.csv")


def trace_rows():
    kt = glob.glob(f"{src}/trace/run_kernel_trace.csv")
    return list(csv.DictReader(open(kt[0]))) if kt else []


# The dominant kernel: the stft_ola kernel with the largest total time in the
# trace; its headline dispatches are the most common grid size among them (the
# bench also times the 8192-stream strong-scaling phase with a larger grid).
rows = [r for r in trace_rows() if "stft_ola" in r["Kernel_Name"]]
tot = collections.Counter()
for r in rows:
    tot[r["Kernel_Name"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
kname = tot.most_common(1)[0][0] if tot else "k_stft_ola"
grids = collections.Counter(r["Grid_Size_X"] for r in rows if r["Kernel_Name"] == kname)
grid = grids.most_common(1)[0][0] if grids else None
ds = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
            if r["Kernel_Name"] == kname and r["Grid_Size_X"] == grid)
med = ds[len(ds) // 2] if ds else None
mn = ds[0] if ds else None
dur = sum(ds) / len(ds) if ds else None
others = sorted({r["Kernel_Name"] for r in rows} - {kname})

# rocprofv3's kernel_stats.csv averages every dispatch of a kernel, and bench.py
# launches the headline kernel at two grids (1024 streams, then the 8192-stream
# strong phase): the same trace split by (kernel, grid), so the headline launch's
# average stands on its own row
by = collections.defaultdict(list)
for r in trace_rows():
    by[(r["Kernel_Name"], r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
if by:
    with open(f"profiles/{tag}_kernel_stats_by_grid.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Grid_Size_X", "Calls", "AverageNs", "MedianNs", "MinNs", "MaxNs", "TotalNs"])
        for (k, g), v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            v = sorted(v)
            w.writerow([k, g, len(v), round(sum(v) / len(v), 1), v[len(v) // 2], v[0], v[-1], sum(v)])


def counters(sub, name):
    """Mean per-dispatch counter values of kernel `name` (prof_driver runs only
    the headline workload, so every dispatch of it is a headline launch)."""
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{src}/{sub}/run_counter_collection.csv"):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] == name:
                per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        for c in per.values():
            for k, v in c.items():
                agg[k].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def hbm_of(p):
    if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
        return (2 * p["FETCH_SIZE"] + p["WRITE_SIZE"]) * 1024
    return None


pmc = {}
for sub in ("fetch", "write", "sq", "lds"):
    pmc.update(counters(sub, kname))
valu_pass = counters("valu", kname)  # its own pass: SQ_INSTS_VALU / GRBM_GUI_ACTIVE again, same launches
for k, v in valu_pass.items():
    pmc.setdefault(k, v)


def valu_issue(p, simds=1024, xcds=8, lanes=64):
    """VALU busy fraction of the dominant kernel from the valu pass: VALU
    cycles per SIMD over the kernel's cycles.  SQ_THREAD_CYCLES_VALU counts
    quad-cycles (4 clocks: one wave64 VALU instruction, packed or not, on a
    16-lane SIMD) times active lanes, summed over the SIMDs: / 64 lanes (full
    waves) x 4 / 1024 SIMDs; it equals SQ_ACTIVE_INST_VALU x 64 here.
    GRBM_GUI_ACTIVE sums the 8 XCDs' clocks.  Also the FP32 flops the counter
    reports (SQ_INSTS_VALU_FLOPS_FP32, per wave instruction: x 64 lanes)."""
    if not {"SQ_THREAD_CYCLES_VALU", "GRBM_GUI_ACTIVE"} <= set(p):
        return None
    kcyc = p["GRBM_GUI_ACTIVE"] / xcds
    busy = p["SQ_THREAD_CYCLES_VALU"] / lanes * 4 / simds
    out = {"valu_cycles_per_simd": busy, "kernel_cycles": kcyc, "busy_frac": busy / kcyc if kcyc else None}
    if "SQ_INSTS_VALU_FLOPS_FP32" in p:
        out["fp32_flops_per_launch"] = p["SQ_INSTS_VALU_FLOPS_FP32"] * lanes
    return out
S, T, N, H = 1024, 480000, 1024, 256
alg_read = S * T * 4
alg_write = S * T * 4
hbm = hbm_of(pmc)
aux = {}
for o in others:
    po = {}
    for sub in ("fetch", "write"):
        po.update(counters(sub, o))
    aux[o] = {"hbm_bytes_per_launch": hbm_of(po), "pmc_per_launch": po}
# bench.py's own HIP-event kernel time from the same profiled run (trace.log)
bench_ms = None
for lf in (f"{src}/trace.log",):
    if os.path.exists(lf):
        for line in open(lf):
            if line.startswith("{"):
                bench_ms = json.loads(line)["roofline"]["kernel_ms"]
out = {
    "tag": tag,
    "workload_key": f"{S}x{T}_N{N}_H{H}",
    "kernel": kname,
    "src_hash": src_hash(),
    "median_duration_ns_trace": med,
    "min_duration_ns_trace": mn,
    "avg_duration_ns_trace": dur,
    "bench_event_ms_same_run": bench_ms,
    "pmc_per_launch": pmc,
    "algorithmic_bytes_per_launch": alg_read + alg_write,
    "hbm_bytes_per_launch": hbm,
    "hbm_over_algorithmic": None if hbm is None else hbm / (alg_read + alg_write),
    "fetch_bytes_corrected": None if "FETCH_SIZE" not in pmc else 2 * pmc["FETCH_SIZE"] * 1024,
    "write_bytes": None if "WRITE_SIZE" not in pmc else pmc["WRITE_SIZE"] * 1024,
    "headline_grid": grid,
    "valu_issue": valu_issue(valu_pass) if valu_pass else None,
    "aux_kernels": aux,
    "note": __doc__.strip(),
}
# the clock the kernel ran at: its cycles (GRBM_GUI_ACTIVE / 8, PMC pass) over its
# average duration in the trace pass of the same lease (the cycle count barely
# moves with the clock: DESIGN.md section 5)
if out["valu_issue"] and dur:
    out["valu_issue"]["clock_ghz"] = out["valu_issue"]["kernel_cycles"] / dur
json.dump(out, open(f"profiles/{tag}_pmc_summary.json", "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k not in ("note", "pmc_per_launch")}, indent=1))
