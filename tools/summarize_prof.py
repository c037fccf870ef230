"""Summarise tools/profile.sh output into profiles/ (run on the CPU side after gpurun
merges gpurun_out/).  Writes

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats of the bench command
  profiles/<tag>_pmc.json           per-leg k_ffd_pipe duration + PMC bytes
  profiles/pmc_latest.json          the same, read by bench.py's roofline

The bench launches k_ffd_pipe for four legs (by_leg below tells them apart by grid size and
dispatch order): config 4 (4096 scenarios), config 2, config 3 and config 5b.
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
# bench.py's k_ffd_pipe launches per leg, in run order (tools/profile.sh: --steps 2 --warmup 1
# --config3-steps 1): config 4 (warmup + steps), config 2 (2 + 10), config 3 (1 + 1), config 5b
# (1 + 1).  Configs 3 and 5b have the same grid (391 segments of 4 stages): they are told apart
# by dispatch order, config 3's launches coming first.
LEGS = [("config4", 4096, 50_000, 5_000), ("config2", 1, 10_000, 1_000), ("config3", 1, 1_000_000, 100_000),
        ("config5", 1, 1_000_000, 100_000)]
N_CONFIG3 = 2


def dominant(rs, dur=None):
    """The rows of the kernel instantiation that did the work: every leg launches the u32 / packed
    k_ffd_pipe pair (fp_pipe_pk.h) with one grid, and the one whose values do not match returns at
    once.  Kept: the name with the largest total duration (trace rows) or the largest counter total."""
    tot = {}
    for r in rs:
        tot[r["Kernel_Name"]] = tot.get(r["Kernel_Name"], 0.0) + (dur(r) if dur else float(r["Counter_Value"]))
    if not tot:
        return rs
    best = max(tot, key=tot.get)
    return [r for r in rs if r["Kernel_Name"] == best]


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def by_leg(rs, grid_key):
    """k_ffd_pipe rows per leg: the largest grid is config 4, the smallest config 2, the
    remaining grid holds config 3 then config 5b in dispatch order."""
    g = {}
    for r in rs:
        if KERNEL in r["Kernel_Name"]:
            g.setdefault(int(r[grid_key]), []).append(r)
    grids = sorted(g, reverse=True)
    out = {}
    if not grids:
        return out
    out["config4"] = g[grids[0]]
    if len(grids) >= 3:
        out["config2"] = g[grids[-1]]
        mid = sorted(g[grids[1]], key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
        out["config3"], out["config5"] = mid[:N_CONFIG3], mid[N_CONFIG3:]
    elif len(grids) == 2:
        out["config3"] = g[grids[1]]
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = glob.glob(os.path.join(base, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        sys.exit(f"no kernel_stats.csv under {base}/trace")
    shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    trace = by_leg(rows(os.path.join(base, "trace", "**", "*kernel_trace.csv")), "Grid_Size_X")
    fetch = by_leg([r for r in rows(os.path.join(base, "fetch", "**", "*counter_collection.csv"))
                    if r["Counter_Name"] == "FETCH_SIZE"], "Grid_Size")
    write = by_leg([r for r in rows(os.path.join(base, "write", "**", "*counter_collection.csv"))
                    if r["Counter_Name"] == "WRITE_SIZE"], "Grid_Size")
    out = {}
    for leg, S, C, N in LEGS:
        tr = trace.get(leg)
        if not tr:
            continue
        tr = dominant(tr, lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        kname = tr[0]["Kernel_Name"]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
        fl = [r for r in fetch.get(leg, []) if r["Kernel_Name"] == kname]
        wl = [r for r in write.get(leg, []) if r["Kernel_Name"] == kname]
        f = statistics.mean(float(r["Counter_Value"]) for r in fl) if fl else None
        w = statistics.mean(float(r["Counter_Value"]) for r in wl) if wl else None
        out[leg] = {
            "kernel": KERNEL, "instantiation": kname, "tag": tag, "S": S, "C": C, "N": N,
            "grid_threads": int(tr[0]["Grid_Size_X"]),
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
