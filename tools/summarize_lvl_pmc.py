"""Summarise tools/lvl_pmc.sh into profiles/<tag>_lvl_pmc.json and profiles/pmc_levelize_latest.json
(read by bench.py's config-5a roofline as `traffic`): the HBM bytes of one levelize call, summed
over its kernels, 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction, MI355X_MICROARCH.md "HBM"),
each counter from its own pass.  A call = one k_lvl_async dispatch; the A1 legacy-order kernels that
tools/lvl_time.py also runs (k_part_*) are left out.
    python tools/summarize_lvl_pmc.py <tag>"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_lvl_zero", "k_indeg_bin", "k_indeg_hist", "k_indeg_check", "k_lvl_prep", "k_edge_hops",
           "k_lvl_async", "k_cs_hist", "k_cs_scan", "k_cs_scatter", "k_cs_pass_late")


def counter(base, name):
    per = {}
    calls = 0
    for p in glob.glob(os.path.join(base, "**", "*counter_collection.csv"), recursive=True):
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != name:
                    continue
                k = next((k for k in KERNELS if k + "(" in r["Kernel_Name"]), None)
                if k is None:
                    continue
                per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
                calls += k == "k_lvl_async"
    return per, calls


def main():
    tag = sys.argv[1]
    base = os.path.join(ROOT, "gpurun_out", f"lvlpmc_{tag}")
    fetch, nf = counter(os.path.join(base, "fetch"), "FETCH_SIZE")
    write, nw = counter(os.path.join(base, "write"), "WRITE_SIZE")
    if not nf or not nw:
        sys.exit("no k_lvl_async dispatches in the counter files")
    kb = 1024.0
    per_kernel = {k: {"fetch_bytes": 2 * fetch.get(k, 0.0) * kb / nf, "write_bytes": write.get(k, 0.0) * kb / nw}
                  for k in KERNELS if k in fetch or k in write}
    for v in per_kernel.values():
        v["hbm_bytes"] = v["fetch_bytes"] + v["write_bytes"]
    out = {"tag": tag, "calls": nf, "workload": "config 5a: levelize the 1M-vertex DAG (tools/lvl_time.py)",
           "hbm_bytes_per_call": sum(v["hbm_bytes"] for v in per_kernel.values()),
           "per_kernel": per_kernel,
           "correction": "hbm_bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (KiB counters); separate --pmc passes"}
    for name in (f"{tag}_lvl_pmc.json", "pmc_levelize_latest.json"):
        with open(os.path.join(ROOT, "profiles", name), "w") as fo:
            json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
