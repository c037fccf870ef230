"""Benchmark: container x node evaluations/s for FFD what-if planning on MI355X.

Headline workload = BASELINE.json configs[3] at its stated size: S = 4096 what-if
scenarios of 50k containers x 5k nodes (ports + anti-affinity + labels, SPEC.md 3
synthetic clusters generated on the device).  Strong scaling: the 4096 scenarios
are split into contiguous blocks, rank r plans 4096/N of them, so N = 1 runs the
whole config on one GPU and SCALE's N = 1 line equals BENCH.

One step = restore the pristine node tables (D2D) + FFD plan of every local
scenario (key sort + placement kernel + packed cost) + all-gather of the packed
costs over RCCL (N > 1) + argmin + hand-off of the winning plan from its owner
rank (one broadcast, N > 1; a D2D copy at N = 1).

value = S_total * C * N / step_time ("work-equivalent" evals/s, SURVEY.md 8(d):
the brute-force container x node count; the kernel prunes most of it).

roofline (dominant kernel k_ffd_pipe): achieved = the launch's essential (algorithmic)
bytes -- 21 B per container + 29 B per node, each read or written once -- / the kernel's
average duration, timed live with HIP events on the launch stream; peak 8000 GB/s.
`traffic` = HBM bytes per launch from rocprofv3 PMC (FETCH_SIZE x 2 gfx950 correction +
WRITE_SIZE, separate passes, profiles/pmc_latest.json), with traffic_over_essential.
The kernel is bound by the latency of the sequential first-fit chain, not by HBM: `latency_model` compares
the measured time with checks x cycles-per-check from the diagnostics build
(profiles/pipe_model_latest.json).  The 16 B x S*C*N figure is reported under
`work_equivalent`, labelled as what it is.

Legs in the same JSON line (rank 0 at N = 1; single scenarios are replicas, they do not shard):
  config1   BASELINE configs[0]: the fleet.kdl dry-run fixtures, microseconds per plan on the GPU
            path and on the single-threaded C oracle, and the "Rust not available" statement
  config2   BASELINE configs[1]: 1 x 10k services x 1k servers (cpu/mem/ports)
  config3   BASELINE configs[2]: 1 x 1M containers x 100k nodes, the north-star sweep
  config5   BASELINE configs[4]: levelize the 1M-vertex depends_on DAG ((V+E)/s, roofline
            on 16V + 12E + 4 bytes), then place its containers on 100k nodes with the levels
  stage2    the scenario-batched feasibility/score sweep against the VALU roofline
  cpu_baseline       the oracle FFD on config-4 scenarios on every usable host core
  cpu_single_thread  the single-threaded C oracle on the same inputs as configs 2, 3 and 5
                     (A1 legacy order, levels, FFD), each GPU result checked bit for bit

    python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus N without an external launcher starts N worker processes itself (before
any GPU call in this parent), one per GPU, over torch.distributed (RCCL).
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

C4, N4, S4, SEED4 = 50_000, 5_000, 4096, 0x5EED0004
C3, N3, SEED3 = 1_000_000, 100_000, 0x5EED0003
C2, N2, SEED2, FLAGS2 = 10_000, 1_000, 0x5EED0002, 1
N5, SEED5 = 100_000, 0x5EED0005
DAG5 = (1000, 500, 50, 10_000, 333)  # chains, chain length, fan-out layers, layer width, 3-cycles
FLAGS = 7
HBM_PEAK_GBPS = 8000.0
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")
# config 5a's HBM bytes per levelize call (tools/lvl_pmc.sh + tools/summarize_lvl_pmc.py)
PMC_LVL_FILE = os.path.join(ROOT, "profiles", "pmc_levelize_latest.json")
MODEL_FILE = os.path.join(ROOT, "profiles", "pipe_model_latest.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scenarios", type=int, default=S4, help="total what-if scenarios (config 4: 4096)")
    ap.add_argument("--config3-steps", type=int, default=3)
    ap.add_argument("--no-legs", action="store_true", help="skip the config 2 / 3 / 5 legs")
    ap.add_argument("--no-stage2", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=12.0, help="CPU baseline sample budget (wall s)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the CPU baseline (default: every usable core, within the cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-launch", action="store_true",
                    help="test hook: each rank prints its rank/world env as JSON and exits (no GPU call)")
    return ap.parse_args()


# ---------------------------------------------------------------------------------------------
# launcher: `python bench.py --gpus N` without torchrun starts N ranks (this parent never
# initialises HIP; each child is a fresh process that binds its own GPU)
# ---------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, poll_s=0.2):
    """Start n rank processes and wait for all of them.  If one exits non-zero (an OOM, an
    FP_E* error, an assertion) the others would block in their next collective forever, so
    they are terminated (then killed) and the launcher exits with the failing rank's code."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code and not rc:
                rc = code
                for q in live:
                    q.terminate()
                deadline = time.time() + 10
                for q in live:
                    try:
                        q.wait(max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
        if live:
            time.sleep(poll_s)
    return rc


# ---------------------------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the oracle FFD on whole config-4 scenarios
# ---------------------------------------------------------------------------------------------
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_quota():
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 CPU quota if any."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return usable, quota, (min(usable, quota) if quota else usable)


def cpu_baseline(budget_s, threads):
    """oracle/fp_oracle.c fpo_place (sort + first-fit scan) on whole 50k x 5k scenarios of
    the same workload, `threads` scenarios at a time on as many host threads (ctypes drops
    the GIL).  1 warm-up wave, then timed waves until ~budget_s (at least 5); the value is
    the median wave rate.  Inputs are generated before the timed waves."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O  # the checker, timed as the CPU baseline only
    O.lib()
    inputs = [O.gen_scenario(SEED4, s, C4, N4, FLAGS) for s in range(threads)]
    singles = []
    for _ in range(3):
        t0 = time.perf_counter()
        O.place(*inputs[0])
        singles.append(C4 * N4 / (time.perf_counter() - t0))
    rates = []
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda i: O.place(*inputs[i]), range(threads)))  # warm-up wave
        t_start = time.perf_counter()
        while len(rates) < 5 or time.perf_counter() - t_start < budget_s:
            t0 = time.perf_counter()
            list(ex.map(lambda i: O.place(*inputs[i]), range(threads)))
            rates.append(threads * C4 * N4 / (time.perf_counter() - t0))
            if len(rates) >= 200:
                break
        wall = time.perf_counter() - t_start
    usable, quota, _ = _cpu_quota()
    return {"value": statistics.median(rates), "unit": "evals/s", "cores": threads, "kind": "port",
            "single_thread_value": statistics.median(singles),
            "nproc": os.cpu_count(), "usable_cpus": usable, "cgroup_cpu_quota": quota, "cpu_model": _cpu_model(),
            "sample": f"{len(rates)} waves of {threads} whole 50k x 5k config-4 scenarios on {threads} host "
                      f"threads (oracle/fp_oracle.c fpo_place: sort + first-fit scan), median wave rate, "
                      f"{wall:.1f} s timed after 1 warm-up wave; single-thread = median of 3 scenarios"}


def _median_ms(fn, reps):
    ts, out = [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts), out


def cpu_single_thread_legs(gpu):
    """the single-threaded C oracle on the same inputs as the GPU legs, timed on
    this host (steady clock; median of 5 after a warm-up where a run is short, one run for the
    ~35 s config-3 / config-5 FFD), and every GPU result checked against it bit for bit:
      A1 legacy order (engine.rs:67-85) and Kahn levels on config 5's DAG, FFD of configs 2, 3
      and 5b.  The two long FFD runs go on two host threads side by side (one core each)."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    from oracle import oracle as O  # checker and CPU baseline only
    O.lib()
    out = {}
    rp, col, hd = gpu["config5"]["graph"]
    O.legacy_order(hd)
    a1_ms, a1_perm = _median_ms(lambda: O.legacy_order(hd), 5)
    g_a1 = gpu["config5"]["legacy"]
    O.levelize(rp, col, hd)
    lv_ms, (el, eo, en) = _median_ms(lambda: O.levelize(rp, col, hd), 5)
    gl, go, gn = gpu["config5"]["levels"]
    lv_ok = bool(np.array_equal(gl, el) and np.array_equal(go, eo) and gn == en)
    V, E = hd.size, col.size
    out["legacy_order_config5"] = {"ms": a1_ms, "unit_value": V / (a1_ms / 1e3), "unit": "vertices/s", "cores": 1,
                                   "gpu_ms_per_step": g_a1["ms_per_step"], "gpu_kernel_ms": g_a1["kernel_ms"],
                                   "gpu_unit_value": g_a1["unit_value"],
                                   "gpu_bit_exact": bool(np.array_equal(g_a1["perm"], a1_perm))}
    out["levelize_config5"] = {"ms": lv_ms, "unit_value": (V + E) / (lv_ms / 1e3), "unit": "(V+E)/s", "cores": 1,
                               "gpu_bit_exact": lv_ok}
    cont2, nodes2 = O.gen_scenario(SEED2, 0, C2, N2, FLAGS2)
    O.place(cont2, nodes2)
    c2_ms, (ea, er, _, _) = _median_ms(lambda: O.place(cont2, nodes2), 5)
    c2_ok = bool(np.array_equal(gpu["config2"]["plan"][0], ea) and np.array_equal(gpu["config2"]["plan"][1], er))
    out["ffd_config2"] = {"ms": c2_ms, "unit_value": C2 * N2 / (c2_ms / 1e3), "unit": "evals/s", "cores": 1,
                          "gpu_bit_exact": c2_ok}

    def long_ffd(name, seed, C, N, level):
        cont, nodes = O.gen_scenario(seed, 0, C, N, FLAGS)
        ms, (ea, er, _, _) = _median_ms(lambda: O.place(cont, nodes, level=level), 1)
        plan = gpu[name]["plan"]
        return name, ms, C * N, bool(np.array_equal(plan[0], ea) and np.array_equal(plan[1], er))

    with ThreadPoolExecutor(2) as ex:
        jobs = [ex.submit(long_ffd, "config3", SEED3, C3, N3, None),
                ex.submit(long_ffd, "config5", SEED5, V, N5, el)]
        for j in jobs:
            name, ms, evals, ok = j.result()
            out[f"ffd_{name}"] = {"ms": ms, "unit_value": evals / (ms / 1e3), "unit": "evals/s", "cores": 1,
                                  "gpu_bit_exact": ok}
    bad = [k for k, v in out.items() if v.get("gpu_bit_exact") is False]
    if bad:
        raise RuntimeError(f"GPU results differ from the oracle: {bad}")
    return out


KDL_FIXTURES = (("readme", "local"), ("hello-world", "default"))  # BASELINE.md config-1 note


def config1_leg(planner, reps=200):
    """BASELINE config 1: the dry-run fixtures (`fleet up local --dry-run`, up.rs:57-136) -- the
    project's fleet.kdl through the KDL front end, then the stage's start order (engine.rs:67-85
    legacy order), Kahn levels and single-host assignment.  GPU = fleetflow_amd.flow.plan_stage
    through the host-pointer C ABI; CPU = the single-threaded C oracle on the same stage graph.
    Both in microseconds per plan (median of `reps` after a warm-up), parity = identical order,
    levels and assignment ("local" for every service: the fixtures list no servers)."""
    import numpy as np

    from fleetflow_amd import flow as F
    from fleetflow_amd.parser import parse_kdl_file
    from oracle import oracle as O  # checker and CPU baseline only
    O.lib()
    out = {}
    for proj, stage in KDL_FIXTURES:
        fl = parse_kdl_file(os.path.join(ROOT, "tests", "golden", "kdl", proj, ".fleetflow", "fleet.kdl"))
        services = list(fl.stages[stage].services)
        plan = F.plan_stage(fl, stage, planner)
        gpu_ms, _ = _median_ms(lambda: F.plan_stage(fl, stage, planner), reps)

        def cpu_plan():
            names, pos2v, rp, col, hd = F.stage_graph(services, fl)
            perm = O.legacy_order(F.has_deps_vector(services, fl))
            lv, _, _ = O.levelize(rp, col, hd)
            return [services[i] for i in perm], [int(lv[v]) for v in pos2v], {n: "local" for n in services}
        cpu_plan()
        cpu_ms, (order, levels, host) = _median_ms(cpu_plan, reps)
        ok = (plan.order == order and [plan.levels[n] for n in services] == levels and not plan.assignment
              and not plan.rejected)
        if not ok:
            raise RuntimeError(f"config 1 ({proj}/{stage}): GPU plan differs from the oracle")
        out[f"{proj}/{stage}"] = {"services": len(services), "order": order, "levels": levels,
                                  "gpu_us_per_plan": gpu_ms * 1e3, "cpu_single_thread_us_per_plan": cpu_ms * 1e3,
                                  "gpu_bit_exact": True, "assignment": "local (no servers in the stage)"}
    import shutil
    cargo = shutil.which("cargo")
    out["rust"] = ("cargo found at " + cargo + "; the Rust crate is not built by the bench") if cargo else \
        "Rust not available; C restatement used (oracle/fp_oracle.c, engine.rs:67-85 restated)"
    out["note"] = ("GPU = KDL front end + stage graph on the host + ONE fp_plan_stage call (k_plan_small: A1 order, "
                   "A2 levels and start order in one kernel, inputs and results in mapped pinned host memory); "
                   "CPU = stage graph + fpo_legacy_order + fpo_levelize, single thread")
    return out


# ---------------------------------------------------------------------------------------------
# roofline helpers
# ---------------------------------------------------------------------------------------------
def _load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def pmc_record(leg, S, C, N):
    """PMC HBM bytes of one k_ffd_pipe launch for this leg, from the committed rocprofv3
    summary (profiles/pmc_latest.json, tools/pmc_summary.py).  Scaled per scenario when
    only the per-scenario count differs (strong-scaled ranks)."""
    d = _load_json(PMC_FILE)
    rec = (d or {}).get(leg)
    if not rec or rec.get("C") != C or rec.get("N") != N:
        return None, None
    b = rec["hbm_bytes_per_launch"]
    if rec.get("S") != S:
        b = b / rec["S"] * S
    return b, rec


def _records(path):
    """The FFD records the timed launches ran (fp_ctx_place_path, read after the timed region)."""
    if not path or not path.get("ran"):
        return None
    return ("packed (cpu, mem) words, fp_pipe_pk.h" if path["packed"] else "u32 fields") + \
        f" (batch OR cpu 0x{path['or_cpu']:x}, mem 0x{path['or_mem']:x})"


def roofline(leg, S, C, N, kernel_s, step_s, path=None):
    """`achieved` / `frac` are ALGORITHMIC: the essential bytes of one launch (every container's
    16 B of demands read once + assign/reason written once, every node's 17 B read once + 12 B
    written back) over the kernel's live-timed duration.  The PMC counter bytes are `traffic`,
    with their ratio to the essential bytes: cutting re-reads lowers that ratio and raises
    nothing artificially."""
    traffic, rec = pmc_record(leg, S, C, N)
    ess = S * (C * 21 + N * 29)  # containers in (16 B) + out (5 B); nodes in (17 B) + back (12 B)
    achieved = ess / kernel_s / 1e9
    out = {"bound": "hbm", "limiter": "latency of the sequential first-fit chain (see latency_model)",
           "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
           "algorithmic_bytes": ess,
           "algorithmic_basis": "21 B per container (cpu, mem, req, conf read; assign u32 + reason u8 written) + "
                                "29 B per node (cpu_free, mem_free, labels, conflict_used u32 + schedulable u8 read; "
                                "three u32 written back), once each per launch",
           "traffic": traffic,
           "traffic_over_essential": traffic / ess if traffic else None,
           "traffic_GBps": traffic / kernel_s / 1e9 if traffic else None,
           "traffic_frac": traffic / kernel_s / 1e9 / HBM_PEAK_GBPS if traffic else None,
           "traffic_source": (f"rocprofv3 PMC {rec.get('tag')}: 2 x FETCH_SIZE + WRITE_SIZE per launch, "
                              f"separate passes (profiles/pmc_latest.json)") if rec else None,
           "kernel": "k_ffd_pipe (fleetflow_amd/csrc/fp_pipe.hip)", "records": _records(path),
           "kernel_ms": kernel_s * 1e3,
           "work_equivalent": {"note": "16 B x S*C*N brute-force evaluations / kernel time: a work count, "
                                       "NOT bandwidth (pruned evaluations never touch memory)",
                               "evals_per_launch": S * C * N,
                               "GBps": 16 * S * C * N / kernel_s / 1e9}}
    m = (_load_json(MODEL_FILE) or {}).get(leg)
    if m and m.get("C") == C and m.get("N") == N:
        lm = dict(m, measured_kernel_ms=kernel_s * 1e3)
        if "slot_cycles_per_scenario" in m:
            lm["model_ms"] = S * m["slot_cycles_per_scenario"] / m["slots"] / (m["clock_ghz"] * 1e6)
        elif "front" in m:
            lm["model_ms"] = m["front"]["model_ms"]
        if traffic:
            lm["hbm_time_at_peak_ms"] = traffic / (HBM_PEAK_GBPS * 1e9) * 1e3
        out["latency_model"] = lm
    return out


# ---------------------------------------------------------------------------------------------
# workers
# ---------------------------------------------------------------------------------------------
def timed(steps, step, sync, barrier):
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    return time.perf_counter() - t0


def single_leg(planner, dev, leg, seed, C, N, flags, steps, warmup, level_t=None):
    """One scenario (a replica per GPU; BASELINE configs 2, 3 and 5b): device-generated inputs
    (SPEC.md 3, the generator of fp_dev_gen_batch), one step = restore the pristine node table +
    dev_place_batch.  Returns the leg's record and its plan (host copies, for the oracle check)."""
    import torch

    from fleetflow_amd import DevBatch
    from fleetflow_amd._lib import FP_K_PLACE, FP_K_SORT
    db = DevBatch.allocate(1, C, N, dev, with_level=level_t is not None)
    planner.dev_gen_batch(seed, db, flags)
    if level_t is not None:
        db.level.copy_(level_t)
    pristine = db.node_snapshot()

    def step():
        db.restore_nodes(pristine)
        planner.dev_place_batch(db)

    for _ in range(max(1, warmup)):
        step()
    torch.cuda.synchronize(dev)
    ref = db.assign.clone()
    planner.profile(True)
    el = timed(steps, step, lambda: torch.cuda.synchronize(dev), lambda: None)
    planner.sync()
    if not torch.equal(db.assign, ref):
        raise RuntimeError(f"{leg}: timed steps did not reproduce the warmup plan")
    k_ms, k_n = planner.kernel_stats(FP_K_PLACE)
    s_ms, s_n = planner.kernel_stats(FP_K_SORT)
    planner.profile(False)
    path = planner.place_path()
    step_s = el / steps
    kernel_s = k_ms / max(k_n, 1) / 1e3
    reason = db.reason.cpu().numpy()
    plan = (db.assign.cpu().numpy().view("uint32"), reason)
    placed = int((reason == 0).sum())
    out = {"value": C * N / step_s, "unit": "evals/s (work-equivalent)", "ms_per_step": step_s * 1e3,
           "steps": steps, "placed": placed, "nofit": int((reason == 1).sum()), "cycle": int((reason == 2).sum()),
           "breakdown_ms": {"ffd_kernel": kernel_s * 1e3, "sort": s_ms / max(s_n, 1)},
           "ns_per_container": step_s / C * 1e9,
           "geometry": planner.geometry(1, C, N),
           "roofline": roofline(leg, 1, C, N, kernel_s, step_s, path)}
    del db, pristine
    torch.cuda.empty_cache()
    return out, plan


def levelize_leg(planner, dev, steps):
    """BASELINE config 5a: Kahn levels of the 1M-vertex depends_on DAG (SPEC.md 3.3: 1000 chains
    x 500, 50 fan-out layers x 10k, 333 injected 3-cycles; host-generated by fleetflow_amd.synth,
    CSR resident in HBM).  Roofline on SURVEY 8(d)'s 16V + 12E + 4 algorithmic bytes."""
    import numpy as np
    import torch

    from fleetflow_amd import synth
    from fleetflow_amd._lib import FP_K_LEVEL
    rp, col, hd = synth.gen_dag(SEED5, *DAG5)
    V, E = hd.size, col.size
    to = lambda a: torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).to(dev)  # noqa: E731
    rp_t, col_t, hd_t = to(rp), to(col), to(hd)
    level_t = torch.empty(V, dtype=torch.int32, device=dev)
    order_t = torch.empty(V, dtype=torch.int32, device=dev)
    ncyc_t = torch.zeros(1, dtype=torch.int32, device=dev)

    def step():
        planner.dev_levelize(rp_t, col_t, hd_t, level_t, order_t, ncyc_t)

    step()
    planner.sync()
    planner.profile(True)
    el = timed(steps, step, lambda: torch.cuda.synchronize(dev), lambda: None)
    planner.sync()
    k_ms, k_n = planner.kernel_stats(FP_K_LEVEL)
    planner.profile(False)
    step_s, kernel_s = el / steps, k_ms / max(k_n, 1) / 1e3
    # A1 (engine.rs:67-85) on the same 1M vertices: fp_dev_legacy_order, timed beside the C
    # restatement's cpu_single_thread.legacy_order_config5 (checked against it there)
    perm_t = torch.empty(V, dtype=torch.int32, device=dev)
    planner.dev_legacy_order(hd_t, perm_t)
    planner.sync()
    planner.profile(True)
    a1_el = timed(steps, lambda: planner.dev_legacy_order(hd_t, perm_t), lambda: torch.cuda.synchronize(dev),
                  lambda: None)
    planner.sync()
    a1_k_ms, a1_k_n = planner.kernel_stats(FP_K_LEVEL)
    planner.profile(False)
    legacy = {"ms_per_step": a1_el / steps * 1e3, "kernel_ms": a1_k_ms / max(a1_k_n, 1), "unit_value": V / (a1_el / steps),
              "unit": "vertices/s", "perm": perm_t.cpu().numpy().view(np.uint32)}
    nbytes = 16 * V + 12 * E + 4
    levels = level_t.cpu().numpy().view(np.uint32)
    pmc = _load_json(PMC_LVL_FILE) or {}
    traffic = pmc.get("hbm_bytes_per_call")
    out = {"workload": "BASELINE config 5a: levelize the 1M-vertex depends_on DAG (deep chains + wide fan-out, "
                       "333 3-cycles)", "V": V, "E": E, "value": (V + E) / step_s, "unit": "(V+E)/s",
           "ms_per_step": step_s * 1e3, "steps": steps, "kernel_ms": kernel_s * 1e3,
           "levels": int(levels[levels != 0xFFFFFFFF].max()) + 1, "cycle_vertices": int(ncyc_t.item()),
           "roofline": {"bound": "hbm", "kernel": "levelizer (k_indeg + k_lvl_async + level sort, fp_order.hip)",
                        "achieved": nbytes / kernel_s / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": nbytes / kernel_s / 1e9 / HBM_PEAK_GBPS, "traffic": traffic,
                        "traffic_over_essential": traffic / nbytes if traffic else None,
                        "traffic_source": (f"rocprofv3 PMC {pmc.get('tag')}: 2 x FETCH_SIZE + WRITE_SIZE summed over "
                                           "the call's kernels, separate passes (profiles/pmc_levelize_latest.json)")
                        if traffic else None,
                        "algorithmic_bytes": nbytes,
                        "limiter": "latency of the longest dependency chain (500 levels of chains)"}}
    return out, (rp, col, hd), level_t, (levels, order_t.cpu().numpy().view(np.uint32), int(ncyc_t.item())), legacy


# VALU lane-operations per container x node evaluation in k_feas's inner loop (no bitmap):
# 62 VALU instructions per 2 nodes x 4 containers per lane (hipcc -S of fp_feas.hip, gfx950)
FEAS_VALU_PER_EVAL = 62 / 8
# peak VALU lane-ops/s: 256 CUs x 4 SIMD x 32 lanes per cycle (wave64 issues over 2 cycles)
# x 2.4 GHz (MI355X_MICROARCH.md)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9


def stage2_leg(planner, dev, steps, S=512):
    """Stage 2 (north_star: 'coalesced containers-by-nodes feasibility and score sweep with
    node-capacity tiles staged in LDS', batched over scenarios): fp_dev_feasibility_batch on
    S config-4 scenarios' pristine node tables -- first feasible node + feasible-node count
    for every (scenario, container).  VALU-bound (every evaluation is computed)."""
    import torch

    from fleetflow_amd import DevBatch
    from fleetflow_amd._lib import FP_K_FEAS
    db = DevBatch.allocate(S, C4, N4, dev)
    planner.dev_gen_batch(SEED4, db, FLAGS)
    first = torch.empty(S * C4, dtype=torch.int32, device=dev)
    count = torch.empty(S * C4, dtype=torch.int32, device=dev)
    planner.dev_feasibility_batch(db, first, count)
    torch.cuda.synchronize(dev)
    ref = count.clone()
    planner.profile(True)
    el = timed(steps, lambda: planner.dev_feasibility_batch(db, first, count),
               lambda: torch.cuda.synchronize(dev), lambda: None)
    planner.sync()
    if not torch.equal(count, ref):
        raise RuntimeError("stage 2: timed steps did not reproduce the warmup sweep")
    k_ms, k_n = planner.kernel_stats(FP_K_FEAS)
    planner.profile(False)
    kernel_s = k_ms / max(k_n, 1) / 1e3
    evals = S * C4 * N4
    rate = evals / kernel_s
    out = {"workload": f"stage-2 feasibility + score sweep, {S} config-4 scenarios x 50k containers x 5k nodes "
                       "(fp_dev_feasibility_batch)",
           "value": evals / (el / steps), "unit": "evals/s", "ms_per_step": el / steps * 1e3, "steps": steps,
           "kernel_ms": kernel_s * 1e3,
           "roofline": {"bound": "valu", "achieved": rate * FEAS_VALU_PER_EVAL / 1e12,
                        "peak": VALU_PEAK_LANE_OPS / 1e12, "unit": "T lane-ops/s",
                        "frac": rate * FEAS_VALU_PER_EVAL / VALU_PEAK_LANE_OPS,
                        "valu_ops_per_eval": FEAS_VALU_PER_EVAL,
                        "note": "every (container, node) pair is evaluated: node tiles are LDS-resident, so "
                                "HBM traffic is ~16 B x (C + N) per scenario plus 8 B of outputs per container"}}
    del db, first, count
    torch.cuda.empty_cache()
    return out


def worker(args):
    if args.dry_launch:
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                          "MASTER_PORT")}), flush=True)
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from fleetflow_amd import DevBatch, Planner, shard
    from fleetflow_amd._lib import FP_K_PLACE, FP_K_SORT

    S_total, C, N = args.scenarios, C4, N4
    shard.check_scenario_ids(S_total)
    base, S = shard.block(rank, world, S_total)
    planner = Planner(local_rank)
    # one dedicated stream for torch's copies/collectives AND the planner kernels
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    planner.set_stream(stream.cuda_stream)
    db = DevBatch.allocate(S, C, N, dev, scen_base=base)
    planner.dev_gen_batch(SEED4, db, FLAGS)
    pristine = db.node_snapshot()
    best = torch.empty(1, dtype=torch.int32, device=dev)
    plan = torch.empty(shard.plan_words(C), dtype=torch.int32, device=dev)
    winner = {}

    def step():
        db.restore_nodes(pristine)
        planner.dev_place_batch(db)
        costs = shard.gather_costs(db.cost, world, S_total) if world > 1 else db.cost
        planner.dev_argmin_cost(costs, best)
        b = int(best.item())  # every rank holds the same winner
        winner["best"] = b
        winner["owner"] = shard.hand_off_plan(b, db.assign, db.reason, C, rank, world, S_total, plan)

    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    ref_cost, ref_plan = db.cost.clone(), plan.clone()
    planner.profile(True)
    elapsed = timed(args.steps, step, lambda: torch.cuda.synchronize(dev), barrier)
    planner.sync()  # raises on a sticky kernel error (e.g. the pipeline's deadlock guard)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    # every timed step re-planned the same inputs: its plans must be bit-identical
    if not torch.equal(db.cost, ref_cost) or not torch.equal(plan, ref_plan):
        raise RuntimeError("timed steps did not reproduce the warmup plan (stream ordering bug?)")
    place_ms, place_n = planner.kernel_stats(FP_K_PLACE)
    sort_ms, sort_n = planner.kernel_stats(FP_K_SORT)
    planner.profile(False)
    path = planner.place_path()
    # per-rank kernel time, max over ranks (the slowest rank sets the step)
    kt = torch.tensor([place_ms / max(place_n, 1), sort_ms / max(sort_n, 1)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(kt, op=dist.ReduceOp.MAX)
    kernel_ms, sort_avg_ms = float(kt[0].item()), float(kt[1].item())

    out = None
    if rank == 0:
        step_s = elapsed / args.steps
        out = {
            "metric": "container x node evaluations/sec (FFD what-if plans, work-equivalent) "
                      "+ achieved GB/s % HBM roofline",
            "value": S_total * C * N / step_s,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_s * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SPEC.md 3, SplitMix64 seed 0x5EED0004, generated on device)",
            "config": {"workload": f"BASELINE config 4: {S_total} what-if scenarios x 50k containers x 5k nodes, "
                                   "ports+anti-affinity+labels; RCCL all-gather of packed costs + argmin + "
                                   "winner plan broadcast from its owner",
                       "scenarios_total": S_total, "scenarios_per_gpu": S, "containers": C, "nodes": N,
                       "parallelism": f"scenario-sharded x{world}"},
            "roofline": roofline("config4", S, C, N, kernel_ms / 1e3, step_s, path),
            "breakdown_ms": {"ffd_kernel": kernel_ms, "sort": sort_avg_ms},
            "best_scenario": winner["best"], "best_owner_rank": winner["owner"],
        }
    # the config-3 leg and the CPU baseline only at N = 1 (single-scenario replicas do not shard)
    if world == 1 and rank == 0:
        del db, pristine
        torch.cuda.empty_cache()
        gpu = {}  # plans of the single-scenario legs, for the oracle check
        if not args.no_legs:
            out["config1"] = dict({"workload": "BASELINE config 1: fleet.kdl dry-run fixtures, depends_on start "
                                               "order + levels + single-host plan, microseconds per plan"},
                                  **config1_leg(planner))
            r, plan = single_leg(planner, dev, "config2", SEED2, C2, N2, FLAGS2, 10, 2)
            gpu["config2"] = {"plan": plan}
            out["config2"] = dict({"workload": "BASELINE config 2: 1 scenario x 10k services x 1k servers, "
                                               "cpu/mem/port constraints"}, **r)
            r, plan = single_leg(planner, dev, "config3", SEED3, C3, N3, FLAGS, args.config3_steps, 1)
            gpu["config3"] = {"plan": plan}
            out["config3"] = dict({"workload": "BASELINE config 3: 1 scenario x 1M containers x 100k nodes, "
                                               "ports+anti-affinity+labels"}, **r)
            lv, graph, level_t, levels, legacy = levelize_leg(planner, dev, 5)
            r, plan = single_leg(planner, dev, "config5", SEED5, graph[2].size, N5, FLAGS, args.config3_steps, 1,
                                 level_t=level_t)
            gpu["config5"] = {"plan": plan, "graph": graph, "levels": levels, "legacy": legacy}
            out["config5"] = {"workload": "BASELINE config 5: levelize the 1M-vertex DAG, then place its 1M "
                                          "containers on 100k nodes (CYCLE members skipped)",
                              "levelize": lv, "place": r,
                              "ms_per_step": lv["ms_per_step"] + r["ms_per_step"]}
            del level_t
            torch.cuda.empty_cache()
        if not args.no_stage2:
            out["stage2"] = stage2_leg(planner, dev, 3)
        if not args.no_cpu_baseline:
            usable, quota, avail = _cpu_quota()
            threads = args.cpu_threads or avail
            out["cpu_baseline"] = cpu_baseline(args.cpu_budget_s, threads)
            if not args.no_legs:
                out["cpu_single_thread"] = cpu_single_thread_legs(gpu)
    if out is not None:
        print(json.dumps(out), flush=True)
    planner.close()
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    worker(args)


if __name__ == "__main__":
    main()
