"""Sweep a context option over device-resident BASELINE workloads: FFD kernel time (HIP
events, median of --reps after one warm-up) per value, and the plan compared with the
first value's (every value must give the same plan).

    python tools/sys_sweep.py --opt systolic --values 0,8,16,32 --loads c3,c4x512,c4x4096
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fleetflow_amd import DevBatch, Planner  # noqa: E402
from fleetflow_amd._lib import FP_K_PLACE, FP_K_SORT  # noqa: E402

LOADS = {"c3": (1, 1_000_000, 100_000, 0x5EED0003), "c2": (1, 10_000, 1_000, 0x5EED0002),
         "c4x512": (512, 50_000, 5_000, 0x5EED0004), "c4x1024": (1024, 50_000, 5_000, 0x5EED0004),
         "c4x2048": (2048, 50_000, 5_000, 0x5EED0004), "c4x4096": (4096, 50_000, 5_000, 0x5EED0004),
         # many small scenarios (the LDS sort's one-workgroup-per-scenario sizing)
         "s4096c6000": (4096, 6_000, 600, 0x5EED0006)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", default="systolic")
    ap.add_argument("--values", default="0,16")
    ap.add_argument("--loads", default="c3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--set", default="", help="extra fixed options name=v,...")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    with Planner(0) as p:
        for kv in filter(None, args.set.split(",")):
            k, v = kv.split("=")
            p.set_option(k, int(v))
        for load in args.loads.split(","):
            S, C, N, seed = LOADS[load]
            db = DevBatch.allocate(S, C, N, dev)
            p.dev_gen_batch(seed, db, 7)
            p.sync()
            snap = db.node_snapshot()
            ref = None
            for v in [int(x) for x in args.values.split(",")]:
                p.set_option(args.opt, v)
                times, walls, sorts = [], [], []
                for r in range(args.reps + 1):
                    db.restore_nodes(snap)
                    torch.cuda.synchronize()
                    p.profile(True)
                    t0 = time.perf_counter()
                    p.dev_place_batch(db)
                    p.sync()
                    w = time.perf_counter() - t0
                    ms, n = p.kernel_stats(FP_K_PLACE)
                    sms, sn = p.kernel_stats(FP_K_SORT)
                    p.profile(False)
                    if r:
                        times.append(ms / max(n, 1))
                        sorts.append(sms / max(sn, 1))
                        walls.append(w * 1e3)
                same = None
                if ref is None:
                    ref = (db.assign.clone(), db.cost.clone())
                else:
                    same = bool(torch.equal(ref[0], db.assign) and torch.equal(ref[1], db.cost))
                # plan digest: equal across library variants when their plans are (tools/ab_variants.sh)
                wts = torch.arange(db.assign.numel(), device=dev, dtype=torch.int64) % 65521 + 1
                digest = int((db.assign.to(torch.int64) * wts).sum().item()) ^ int(db.cost.sum().item())
                del wts
                print(json.dumps({"load": load, "S": S, "C": C, "N": N, "opt": args.opt, "value": v, "digest": digest,
                                  "ffd_ms": round(statistics.median(times), 3),
                                  "sort_ms": round(statistics.median(sorts), 3),
                                  "wall_ms": round(statistics.median(walls), 3), "same_plan": same,
                                  "geometry": p.geometry(S, C, N)}), flush=True)
            p.set_option(args.opt)
            del db, snap, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
