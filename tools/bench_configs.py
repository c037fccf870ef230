"""Timings of BASELINE configs 2, 3 and 5 on one MI355X (device-resident inputs,
warm medians of the wall time per call and of the HIP-event kernel times of the same
calls), next to the single-thread C oracle
on the same inputs (checker + CPU baseline).  Writes one JSON line per config.

    python tools/bench_configs.py [--reps 3] [--no-cpu]

Config 4 is bench.py's workload.  Every GPU result is compared bit-for-bit with
the oracle's before its time is reported.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import DevBatch, Planner  # noqa: E402
from fleetflow_amd._lib import FP_K_FEAS, FP_K_LEVEL, FP_K_PLACE, FP_K_SORT  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker / CPU baseline only)

SEED = 0x5EED0000


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32 if a.dtype == np.uint32 else a.dtype)).to(dev)


def dev_batch_from(cont, nodes, dev, level=None):
    C, N = len(cont[0]), len(nodes[0])
    db = DevBatch.allocate(1, C, N, dev, with_level=level is not None)
    for t, a in zip((db.cpu, db.mem, db.req, db.conf), cont):
        t.copy_(to_dev(np.asarray(a, np.uint32), dev))
    for t, a in zip((db.cf, db.mf, db.lab, db.cu), nodes[:4]):
        t.copy_(to_dev(np.asarray(a, np.uint32), dev))
    db.sched.copy_(torch.from_numpy(np.asarray(nodes[4], np.uint8)).to(dev))
    if level is not None:
        db.level.copy_(to_dev(np.asarray(level, np.uint32), dev))
    return db


def warm_median(p, call, kids, reps, before=None):
    """One untimed warm-up call, then `reps` timed calls: the median wall time and, per kernel
    id, the median of the per-call HIP-event times (each call's own launches), so that a
    kernel time never includes the cold first call and never exceeds its wall."""
    if before:
        before()
    call()
    p.sync()
    for k in kids:  # drain the warm-up's pending event pairs (if profiling was on)
        p.kernel_stats(k)
    walls, ev = [], {k: [] for k in kids}
    for _ in range(reps):
        if before:
            before()
        torch.cuda.synchronize()
        p.profile(False)
        p.profile(True)
        t0 = time.perf_counter()
        call()
        p.sync()
        walls.append(time.perf_counter() - t0)
        for k in kids:
            ms, n = p.kernel_stats(k)
            ev[k].append(ms)  # the call's total event time for this kernel id
    p.profile(False)
    print("walls (ms):", [round(w * 1e3, 3) for w in walls], {k: [round(x, 3) for x in v] for k, v in ev.items()},
          file=sys.stderr)
    return statistics.median(walls) * 1e3, {k: statistics.median(v) for k, v in ev.items()}


def time_place(p, db, reps):
    snap = db.node_snapshot()
    wall, ev = warm_median(p, lambda: p.dev_place_batch(db), (FP_K_PLACE, FP_K_SORT), reps,
                           before=lambda: db.restore_nodes(snap))
    return wall, ev[FP_K_PLACE], ev[FP_K_SORT]


def check_plan(db, ea, er):
    got_a = db.assign.cpu().numpy().view(np.uint32)
    got_r = db.reason.cpu().numpy()
    return bool(np.array_equal(got_a, ea) and np.array_equal(got_r, er))


def cpu_time(fn):
    t0 = time.perf_counter()
    out = fn()
    return out, (time.perf_counter() - t0) * 1e3


def ffd_config(p, dev, name, seed, C, N, flags, reps, cpu, level=None):
    cont, nodes = O.gen_scenario(seed, 0, C, N, flags)
    db = dev_batch_from(cont, nodes, dev, level)
    wall_ms, kern_ms, sort_ms = time_place(p, db, reps)
    (ea, er, _, _), cpu_ms = cpu_time(lambda: O.place(cont, nodes, level=level))
    ok = check_plan(db, ea, er)
    evals = C * N
    out = {"config": name, "C": C, "N": N, "flags": flags, "bit_exact": ok,
           "gpu_wall_ms": wall_ms, "ffd_kernel_ms": kern_ms, "sort_ms": sort_ms,
           "work_equiv_evals_per_s": evals / (wall_ms / 1e3),
           "placed": int((er == 0).sum()), "nofit": int((er == 1).sum()), "cycle": int((er == 2).sum())}
    if cpu:
        out.update({"cpu_oracle_ms": cpu_ms, "cpu_cores": 1, "speedup_vs_cpu": cpu_ms / wall_ms})
    return out


def levelize_config(p, dev, reps, cpu):
    rp, col, hd = O.gen_dag(SEED + 5, 1000, 500, 50, 10_000, 333)
    V, E = hd.size, col.size
    rp_t, col_t = to_dev(rp, dev), to_dev(col, dev)
    hd_t = torch.from_numpy(hd).to(dev)
    level_t = torch.empty(V, dtype=torch.int32, device=dev)
    order_t = torch.empty(V, dtype=torch.int32, device=dev)
    ncyc_t = torch.zeros(1, dtype=torch.int32, device=dev)
    wall, ev = warm_median(p, lambda: p.dev_levelize(rp_t, col_t, hd_t, level_t, order_t, ncyc_t), (FP_K_LEVEL,), reps)
    (el, eo, en), cpu_ms = cpu_time(lambda: O.levelize(rp, col, hd))
    ok = (np.array_equal(level_t.cpu().numpy().view(np.uint32), el) and
          np.array_equal(order_t.cpu().numpy().view(np.uint32), eo) and int(ncyc_t.item()) == en)
    wall /= 1e3
    out = {"config": "5a: levelize 1M-vertex DAG", "V": V, "E": E, "levels": int(el[el != 0xFFFFFFFF].max()) + 1,
           "cycle_vertices": en, "bit_exact": bool(ok), "gpu_wall_ms": wall * 1e3, "levelize_gpu_ms": ev[FP_K_LEVEL],
           "vertices_edges_per_s": (V + E) / wall,
           "algorithmic_bytes": 16 * V + 12 * E + 4,
           "achieved_GBps": (16 * V + 12 * E + 4) / wall / 1e9}
    if cpu:
        out.update({"cpu_oracle_ms": cpu_ms, "cpu_cores": 1, "speedup_vs_cpu": cpu_ms / (wall * 1e3)})
    return out, el


def feas_config(p, dev, name, seed, C, N, reps, cpu, bitmap):
    """Stage-2 sweep (fp_dev_feasibility) on the pristine node table of a config."""
    cont, nodes = O.gen_scenario(seed, 0, C, N, 7)
    db = dev_batch_from(cont, nodes, dev)
    first_t = torch.empty(C, dtype=torch.int32, device=dev)
    count_t = torch.empty(C, dtype=torch.int32, device=dev)
    bm_t = torch.empty(((C + 63) // 64) * N, dtype=torch.int64, device=dev) if bitmap else None
    wall, ev = warm_median(p, lambda: p.dev_feasibility(db, first_t, count_t, bm_t), (FP_K_FEAS,), reps)
    kern_ms = ev[FP_K_FEAS]
    out = {"config": name, "C": C, "N": N, "bitmap": bitmap, "gpu_wall_ms": wall, "feas_kernel_ms": kern_ms,
           "evals_per_s": C * N / (kern_ms / 1e3), "work_equiv_GBps": 16 * C * N / (kern_ms / 1e3) / 1e9,
           "bitmap_GBps": (((C + 63) // 64) * N * 8 / (kern_ms / 1e3) / 1e9) if bitmap else 0.0}
    if cpu:
        # checker on a sample of containers (the full C x N sweep is minutes of CPU time)
        k = min(C, 2000)
        sub = tuple(np.asarray(a)[:k] for a in cont)
        (ef, ec, _), cpu_ms = cpu_time(lambda: O.feasibility(sub, nodes, want_bitmap=False))
        ok = (np.array_equal(first_t[:k].cpu().numpy().view(np.uint32), ef) and
              np.array_equal(count_t[:k].cpu().numpy().view(np.uint32), ec))
        out.update({"bit_exact_sample": bool(ok), "cpu_oracle_evals_per_s": k * N / (cpu_ms / 1e3), "cpu_cores": 1})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", default="2,3,5,f")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cpu = not args.no_cpu
    only = set(args.only.split(","))
    with Planner(0) as p:
        _opts.apply_env(p)
        if "2" in only:
            print(json.dumps(ffd_config(p, dev, "2: 10k services x 1k servers, cpu/mem/ports", SEED + 2,
                                        10_000, 1_000, 1, args.reps, cpu)), flush=True)
        if "3" in only:
            print(json.dumps(ffd_config(p, dev, "3: 1M containers x 100k nodes, labels + anti-affinity",
                                        SEED + 3, 1_000_000, 100_000, 7, args.reps, cpu)), flush=True)
        if "l" in only:  # levelization alone
            print(json.dumps(levelize_config(p, dev, args.reps, cpu)[0]), flush=True)
        if "5" in only:
            lv, level = levelize_config(p, dev, args.reps, cpu)
            print(json.dumps(lv), flush=True)
            print(json.dumps(ffd_config(p, dev, "5b: place the DAG's 1M containers on 100k nodes (CYCLE skipped)",
                                        SEED + 5, level.size, 100_000, 7, args.reps, cpu, level=level)),
                  flush=True)
        if "f" in only:
            print(json.dumps(feas_config(p, dev, "stage 2 sweep, config-2 shape", SEED + 2, 10_000, 1_000,
                                         args.reps, cpu, True)), flush=True)
            print(json.dumps(feas_config(p, dev, "stage 2 sweep, config-3 shape (no bitmap)", SEED + 3,
                                         1_000_000, 100_000, args.reps, cpu, False)), flush=True)
            print(json.dumps(feas_config(p, dev, "stage 2 sweep, 250k x 100k with bitmap", SEED + 3,
                                         250_000, 100_000, args.reps, cpu, True)), flush=True)


if __name__ == "__main__":
    main()
