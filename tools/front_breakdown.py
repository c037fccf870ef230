"""Where a placement's cycles go at the FFD front, from the diagnostics build's
per-batch timeline (tools/pipe_stats.py TIMELINE=...; scenario 0, global stages 0-15).

Per batch i of a stage: wait = input available - loop top (spinning on the upstream ring / link),
input = read done - available, prescan = prescan end - read done, group = group loop end - prescan end
(exact checks, systolic fill, re-tests, mask upkeep), forward = next loop top - group loop end
(assignment stores, forwarding, output-ring waits).  "Filling" batches place >= FILL of their valid
containers (and hold >= 32): the stage is then the front (its group fills for the stream's current sizes);
the wait before the first batch of a run of filling batches is the front's travel to the stage, not
counted.

    python tools/front_breakdown.py tl.csv [clock_ghz] [FILL]"""
import json
import sys

import numpy as np
import pandas as pd


def breakdown(path, ghz=2.4, fill=0.25):
    d = pd.read_csv(path).sort_values(["stage", "batch"])
    out = {"file": path, "clock_ghz": ghz, "fill_threshold": fill, "stages": {}}
    tot = {k: 0.0 for k in ("wait", "input", "prescan", "group", "forward")}
    tot_hits = tot_batches = 0
    for st, g in d.groupby("stage"):
        g = g.reset_index(drop=True)
        nxt = g.t_top.shift(-1)
        ph = pd.DataFrame({"wait": g.t_avail - g.t_top, "input": g.t_in - g.t_avail, "prescan": g.t_pre - g.t_in,
                           "group": g.t_cand - g.t_pre, "forward": nxt - g.t_cand})
        ok = nxt.notna() & (g.valid > 0)
        front = ok & (g.hits >= fill * g.valid) & (g.hits > 0) & (g.valid >= 32)
        # a run of filling batches: the wait before its first batch is the time the front took to
        # reach this stage, not a stall of the fill
        first_of_run = front & ~front.shift(1, fill_value=False)
        ph.loc[first_of_run, "wait"] = 0
        h = int(g.hits[front].sum())
        rec = {"batches": int(ok.sum()), "front_batches": int(front.sum()), "front_hits": h,
               "hits_all": int(g.hits.sum()), "checks_front": int(g.checks[front].sum())}
        if h:
            rec["cyc_per_placement"] = {k: float(ph[k][front].sum() / h) for k in ph}
            rec["cyc_per_placement"]["total"] = float(sum(rec["cyc_per_placement"].values()))
            rec["cyc_per_front_batch"] = {k: float(ph[k][front].mean()) for k in ph}
            rec["hits_per_front_batch"] = h / int(front.sum())
            for k in tot:
                tot[k] += float(ph[k][front].sum())
            tot_hits += h
            tot_batches += int(front.sum())
        out["stages"][int(st)] = rec
    if tot_hits:
        out["front_cyc_per_placement"] = {k: v / tot_hits for k, v in tot.items()}
        out["front_cyc_per_placement"]["total"] = sum(tot.values()) / tot_hits
        out["front_cyc_per_batch"] = {k: v / tot_batches for k, v in tot.items()}
        out["front_hits_per_batch"] = tot_hits / tot_batches
        busy = tot["input"] + tot["prescan"] + tot["group"] + tot["forward"]
        out["front_share_of_busy"] = {k: tot[k] / busy for k in ("input", "prescan", "group", "forward")}
    return out


if __name__ == "__main__":
    ghz = float(sys.argv[2]) if len(sys.argv) > 2 else 2.4
    fill = float(sys.argv[3]) if len(sys.argv) > 3 else 0.25
    r = breakdown(sys.argv[1], ghz, fill)
    print(json.dumps({k: v for k, v in r.items() if k != "stages"}, indent=1))
    for st, rec in r["stages"].items():
        c = rec.get("cyc_per_placement")
        if c:
            print(f"stage {st:2d}: front batches {rec['front_batches']:5d} hits {rec['front_hits']:7d} "
                  f"({rec['hits_per_front_batch']:.1f}/batch)  cyc/placement " +
                  " ".join(f"{k} {v:6.0f}" for k, v in c.items()))
