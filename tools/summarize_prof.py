"""Summarise tools/profile.sh output into profiles/ (run on the CPU side after gpurun
merges gpurun_out/).  Writes

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats of the bench command
  profiles/<tag>_pmc.json           per-leg k_ffd_pipe duration + PMC bytes
  profiles/pmc_latest.json          the same, read by bench.py's roofline

The bench launches k_ffd_pipe for two legs with different grids: config 4 (4096
scenarios: the largest grid) and config 3 (one 1M x 100k scenario).  Dispatches are
grouped by grid size; the largest grid is config 4, the next config 3.
HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE counts half the bytes of
wide coalesced reads, MI355X_MICROARCH.md "HBM"), each counter from its own --pmc pass."""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_ffd_pipe"
LEGS = [("config4", 4096, 50_000, 5_000), ("config3", 1, 1_000_000, 100_000)]


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def by_grid(rs, grid_key):
    g = {}
    for r in rs:
        if KERNEL in r["Kernel_Name"]:
            g.setdefault(int(r[grid_key]), []).append(r)
    return [g[k] for k in sorted(g, reverse=True)]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = glob.glob(os.path.join(base, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        sys.exit(f"no kernel_stats.csv under {base}/trace")
    shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    trace = by_grid(rows(os.path.join(base, "trace", "**", "*kernel_trace.csv")), "Grid_Size_X")
    fetch = by_grid([r for r in rows(os.path.join(base, "fetch", "**", "*counter_collection.csv"))
                     if r["Counter_Name"] == "FETCH_SIZE"], "Grid_Size")
    write = by_grid([r for r in rows(os.path.join(base, "write", "**", "*counter_collection.csv"))
                     if r["Counter_Name"] == "WRITE_SIZE"], "Grid_Size")
    out = {}
    for i, (leg, S, C, N) in enumerate(LEGS):
        if i >= len(trace):
            break
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace[i]]
        f = statistics.mean(float(r["Counter_Value"]) for r in fetch[i]) if i < len(fetch) else None
        w = statistics.mean(float(r["Counter_Value"]) for r in write[i]) if i < len(write) else None
        out[leg] = {
            "kernel": KERNEL, "tag": tag, "S": S, "C": C, "N": N,
            "grid_threads": int(trace[i][0]["Grid_Size_X"]),
            "launches_traced": len(durs),
            "avg_duration_ms": statistics.mean(durs) / 1e6,
            "fetch_size_kb": f, "write_size_kb": w,
            "fetch_bytes": 2 * f * 1024 if f is not None else None,
            "write_bytes": w * 1024 if w is not None else None,
            "hbm_bytes_per_launch": (2 * f + w) * 1024 if f is not None and w is not None else None,
            "correction": "hbm_bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (FETCH_SIZE/WRITE_SIZE in KiB); "
                          "separate --pmc passes",
        }
    for name in (f"{tag}_pmc.json", "pmc_latest.json"):
        with open(os.path.join(ROOT, "profiles", name), "w") as fo:
            json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
