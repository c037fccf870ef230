"""Summarise tools/profile.sh output into profiles/ (run on the CPU side after gpurun
merges gpurun_out/).  Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats),
profiles/<tag>_pmc.json and profiles/pmc_ffd_latest.json (read by bench.py)."""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_ffd_pipe"


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = glob.glob(os.path.join(base, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        sys.exit(f"no kernel_stats.csv under {base}/trace")
    shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    trace = rows(os.path.join(base, "trace", "**", "*kernel_trace.csv"))
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace if KERNEL in r["Kernel_Name"]]

    def counter(kind, name):
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(base, kind, "**", "*counter_collection.csv"))
                if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
        return statistics.mean(vals) if vals else None

    fetch = counter("fetch", "FETCH_SIZE")
    write = counter("write", "WRITE_SIZE")
    d = {
        "kernel": KERNEL, "tag": tag, "scenarios_per_launch": 512, "C": 50000, "N": 5000,
        "launches_traced": len(durs),
        "avg_duration_ms": statistics.mean(durs) / 1e6 if durs else None,
        "fetch_size_kb": fetch, "write_size_kb": write,
        # gfx950: FETCH_SIZE reports half the bytes of a wide coalesced read (MI355X_MICROARCH.md HBM)
        "hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None else None,
        "correction": "hbm_bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024; separate --pmc passes",
    }
    for name in (f"{tag}_pmc.json", "pmc_ffd_latest.json"):
        with open(os.path.join(ROOT, "profiles", name), "w") as f:
            json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
