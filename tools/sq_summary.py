"""Summarise tools/pmc_sq.sh output: per-dispatch averages of every counter for one kernel."""
import collections
import csv
import glob
import sys

tag, kern = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_ffd")
for p in sorted(glob.glob(f"gpurun_out/sq_{tag}/p*/**/*counter_collection.csv", recursive=True)):
    agg, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(p)):
        if kern not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    n = max(len(disp), 1)
    print(p.split("/")[2], {k: f"{v / n:.4g}" for k, v in sorted(agg.items())})
