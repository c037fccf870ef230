"""Latency model of k_ffd_pipe from the diagnostics build (per-stage s_memtime
counters, libfleetplace_stats.so) for both bench legs.  Writes the JSON that
bench.py's roofline reports as `latency_model` (profiles/pipe_model_latest.json)
plus the raw per-stage counters.

    python tools/pipe_model.py [out.json]     (on the GPU box; builds nothing)

config 4 (many scenarios, throughput-bound): every scenario's B segments each hold one
of the device's resident segment slots (occupancy x CUs, fp_debug_pipe_geom) for the
segment's lifetime (s_memtime from its start to the end of its stream).  With lag = S
the segments of a scenario run phase by phase, so
    model_ms = S x sum_b life_b / slots / clock
and the busy share of a lifetime is the exact checks + prescans; the rest is input
waits, forwarding and the per-batch bookkeeping.
config 3 (one scenario, one-group stages): every container walks the stages in FFD order
until a node of the stage fits it.  Reported: container-stage visits, exact checks,
placements and the summed busy cycles over the launch's cycles (the average number of
stages busy at once) -- the chain of exact checks at the placement frontier, not memory,
sets the time.
"""
import ctypes as ct
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FLEETPLACE_LIB", os.path.join(ROOT, "fleetflow_amd", "libfleetplace_stats.so"))

import torch  # noqa: E402

import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import DevBatch, Planner, _lib  # noqa: E402

# (leg, scenarios in the diagnostics run, C, N, seed)
LEGS = [("config4", int(os.environ.get("S_DIAG", 4096)), 50_000, 5_000, 0x5EED0004),
        ("config3", 1, 1_000_000, 100_000, 0x5EED0003)]


def geom(p, S, C, N):
    g = p.geometry(S, C, N)  # fp_place_geometry (the product ABI)
    return {"G": g["groups"], "W": g["stages"], "B": g["segments"], "R": g["ring"], "lag": g["lag"],
            "link_slots": g["link_slots"], "bounded": g["bounded"], "resident_segments": g["resident"],
            "systolic": g["systolic"]}


def clock_ghz(p):
    L = _lib.load()
    f = L.fp_debug_clock_ghz
    f.argtypes = [ct.c_void_p, ct.POINTER(ct.c_double)]
    v = ct.c_double()
    assert f(p._ctx, ct.byref(v)) == 0
    return v.value


def measure(p, S, C, N, seed):
    db = DevBatch.allocate(S, C, N, "cuda:0")
    p.dev_gen_batch(seed, db, 7)
    p.sync()
    pristine = db.node_snapshot()
    torch.cuda.synchronize()
    L = _lib.load()
    f = L.fp_debug_pipe_stats
    f.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
    buf = (ct.c_ulonglong * 256)()
    p.profile(False)
    p.profile(True)
    for _ in range(2):
        db.restore_nodes(pristine)
        torch.cuda.synchronize()
        f(buf, 1)
        p.dev_place_batch(db)
        p.sync()
    ms, n = p.kernel_stats(_lib.FP_K_PLACE)
    placed = int((db.reason == 0).sum().item())
    f(buf, 0)
    v = [[buf[w * 16 + i] for i in range(16)] for w in range(16)]
    del db, pristine
    torch.cuda.empty_cache()
    return ms / n, placed, [r for r in v if any(r)]  # counters of the last launch (reset before it)


def front_model(p, kms):
    """Config 3: per-stage spans of scenario 0 (fp_debug_stage_span, filled by the launch that
    measure() just ran).  The first container reaches stage j at ~ j x front_us_per_stage:
    stage j - 1 forwards only once its group is full for the stream's current sizes, and it
    fills its group by serial exact checks -- so the launch is the time for that front to
    cross every stage plus the last stages' drain."""
    L = _lib.load()
    f = L.fp_debug_stage_span
    f.argtypes = [ct.POINTER(ct.c_ulonglong)]
    buf = (ct.c_ulonglong * (4096 * 8))()
    f(buf)
    rows = [[buf[i * 8 + k] for k in range(8)] for i in range(4096)]
    rows = [r for r in rows if r[0]]
    t0 = min(r[0] for r in rows)
    first = [(r[1] - t0) / 100.0 for r in rows]  # us (s_memrealtime, 100 MHz)
    end = [(r[2] - t0) / 100.0 for r in rows]
    n = len(rows)
    lo, hi = n // 10, n - 1  # slope of the front past the start-up
    slope = (first[hi] - first[lo]) / (hi - lo)
    return {"stages_traced": n, "front_us_per_stage": slope, "first_input_last_stage_us": first[-1],
            "last_stage_drain_us": end[-1] - first[-1], "launch_end_us": max(end),
            "model_ms": (slope * n + (end[-1] - first[-1])) / 1e3, "placements_per_stage": sum(r[7] for r in rows) / n,
            "formula": "kernel_ms ~ front_us_per_stage x stages + last-stage drain: stage j - 1 forwards its first "
                       "container once its group is full for the stream's sizes, so the groups fill one after another "
                       "by serial exact checks (~175 cycles each) -- the launch is bound by that front, not by memory"}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pipe_model.json")
    p = Planner(0)
    _opts.apply_env(p)
    clk = clock_ghz(p)
    latest, raw = {}, {"clock_ghz": clk}
    for leg, S, C, N, seed in LEGS:
        g = geom(p, S, C, N)
        kms, placed, v = measure(p, S, C, N, seed)
        per = lambda i: sum(r[i] for r in v) / S  # noqa: E731  per scenario
        checks, hits, visits = per(1), per(2), per(0)
        busy = per(9) + per(10)
        raw[leg] = {"geometry": g, "kernel_ms_diag_build": kms, "placed": placed,
                    "per_stage_slot": [{"visits": r[0] / S, "checks": r[1] / S, "hits": r[2] / S, "batches": r[3] / S,
                                        "input_Mcycles": r[8] / S / 1e6, "prescan_Mcycles": r[9] / S / 1e6,
                                        "cand_Mcycles": r[10] / S / 1e6, "fwd_Mcycles": r[11] / S / 1e6,
                                        "out_wait_Mcycles": r[12] / S / 1e6, "life_Mcycles": r[13] / S / 1e6}
                                       for r in v]}
        m = {"C": C, "N": N, "S_diag": S, "source": "tools/pipe_model.py, diagnostics build (libfleetplace_stats.so)",
             "geometry": g, "clock_ghz": clk, "kernel_ms_diag_build": kms,
             "container_stage_visits_per_scenario": visits, "checks_per_scenario": checks,
             "placements_per_scenario": hits, "busy_cycles_per_scenario": busy,
             "cycles_per_check": per(10) / max(checks, 1)}
        if leg == "config4":
            life = [r[13] / S for r in v]  # stats slot = segment b (B x W <= 16)
            slots = g["resident_segments"]
            m.update({"segments": g["B"], "slots": slots, "segment_life_cycles": life,
                      "slot_cycles_per_scenario": sum(life), "busy_share": busy / max(sum(life), 1),
                      "formula": "kernel_ms = S x slot_cycles_per_scenario / slots / clock: every scenario holds one "
                                 "of the device's resident segment slots per segment for the segment's lifetime "
                                 "(lag = S: segment b of every scenario runs after segment b-1's phase), busy with "
                                 "exact checks / prescans for busy_share of it",
                      "model_ms_diag": S * sum(life) / slots / (clk * 1e6)})
        else:
            m["front"] = front_model(p, kms)
            launch_cycles = kms * 1e-3 * clk * 1e9
            m.update({"segments": g["B"], "stages": g["B"] * g["W"],
                      "stages_busy_on_average": busy / launch_cycles,
                      "note": "one scenario: every container walks the one-group stages in FFD order until a node fits "
                              "(visits per container = container_stage_visits / C); the summed busy cycles over the "
                              "launch's cycles give the stages busy at once -- the chain of exact checks at the "
                              "placement frontier sets the time, not memory"})
        latest[leg] = m
        print(leg, json.dumps(m), flush=True)
    with open(out_path, "w") as fo:
        json.dump(latest, fo, indent=1)
    with open(out_path.replace(".json", "_raw.json"), "w") as fo:
        json.dump(raw, fo, indent=1)


if __name__ == "__main__":
    main()
