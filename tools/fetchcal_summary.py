"""Summarise tools/fetchcal.sh: per calibration kernel, FETCH_SIZE and WRITE_SIZE (KiB, from
rocprofv3's counter_collection.csv) against the bytes the kernel moves, and the factor
bytes / counter bytes.  Writes profiles/<tag>_fetchcal.json."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(k, ctr):
    vals = []
    for p in glob.glob(os.path.join(ROOT, "gpurun_out", "fetchcal", f"{k}_{ctr}", "**", "*counter_collection.csv"),
                       recursive=True):
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                if r["Counter_Name"] == ctr and name.split("(")[0].strip().endswith(k):
                    vals.append(float(r["Counter_Value"]))
    return sum(vals) * 1024 if vals else None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
    out = {}
    for k in ("r4", "r16", "g4", "w4", "w1", "w16"):
        log = os.path.join(ROOT, "gpurun_out", "fetchcal", f"{k}_FETCH_SIZE.log")
        nbytes = None
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{"):
                    nbytes = json.loads(line)["bytes"]
        fb, wb = counter(k, "FETCH_SIZE"), counter(k, "WRITE_SIZE")
        moved = fb if k[0] in "rg" else wb
        out[k] = {"bytes": nbytes, "fetch_size_bytes": fb, "write_size_bytes": wb,
                  "factor": (nbytes / moved) if (nbytes and moved) else None}
    with open(os.path.join(ROOT, "profiles", f"{tag}_fetchcal.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
