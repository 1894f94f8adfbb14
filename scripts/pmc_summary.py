"""Average PMC counters per dispatch of a kernel from gpurun_out/pmc/p*/ CSVs."""
import collections
import csv
import glob
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "stft_ola_fused"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    for c in per.values():
        for k, v in c.items():
            agg[k].append(v)
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):.4e}")
