"""Summarise tools/pmc_sq.sh output: per-dispatch averages of every counter for one kernel."""
import collections
import csv
import glob
import sys

tag, kern = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_ffd")
for p in sorted(glob.glob(f"gpurun_out/sq_{tag}/p*/**/*counter_collection.csv", recursive=True)):
    agg, disp = collections.defaultdict(float), set()
    rs = [r for r in csv.DictReader(open(p)) if kern in r["Kernel_Name"]]
    # the u32 / packed pair: keep the instantiation with the most wave cycles (the other returns at once)
    by = collections.defaultdict(float)
    for r in rs:
        by[r["Kernel_Name"]] += float(r["Counter_Value"]) if r["Counter_Name"] in ("SQ_WAVE_CYCLES", "SQ_INSTS") else 0.0
    if by:
        top = max(by, key=by.get)
        rs = [r for r in rs if r["Kernel_Name"] == top]
        print(p.split("/")[2], "kernel", top[:90])
    for r in rs:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    n = max(len(disp), 1)
    print(p.split("/")[2], {k: f"{v / n:.4g}" for k, v in sorted(agg.items())})
