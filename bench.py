"""Benchmark: container x node evaluations/s for FFD what-if planning on MI355X.

Workload (BASELINE.json configs[3], sharded weak): every rank plans S_LOCAL=512
independent what-if scenarios of 50k containers x 5k nodes (SPEC.md section 3
synthetic clusters, generated on the device), so --gpus 8 runs exactly config
4's 4096 scenarios.  One step = restore the pristine node tables (D2D copy) +
FFD plan of every local scenario (key sort + placement kernel + packed cost) +
one all-gather of the packed costs over RCCL (N>1) + the global argmin.

value = S_total * C * N / step_time  ("work-equivalent" evals: SURVEY.md 8(d)).
roofline.achieved = 16 B x (S_local*C*N) / average FFD-kernel duration, measured
with HIP events on the launch stream (16 B per container x node
evaluation); peak = 8000 GB/s HBM (MI355X_MICROARCH.md).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

C_PER_SCEN = 50_000
N_PER_SCEN = 5_000
S_LOCAL = 512
SEED = 0x5EED0004
FLAGS = 7
HBM_PEAK_GBPS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scenarios-per-gpu", type=int, default=S_LOCAL)
    ap.add_argument("--cpu-budget-s", type=float, default=15.0, help="CPU baseline sample budget (wall s)")
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                    help="host threads for the CPU baseline (the GPU box grants 16 per GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(budget_s, threads):
    """Oracle FFD (oracle/fp_oracle.c) on a bounded sample of the same workload:
    whole scenarios of rank 0's shard, one per host thread at a time (the C calls
    release the GIL), until ~budget_s of wall time.  Also reports the
    single-thread rate measured on the first scenario."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O  # the checker, timed as the CPU baseline only
    O.lib()
    inputs = [O.gen_scenario(SEED, s, C_PER_SCEN, N_PER_SCEN, FLAGS) for s in range(threads)]
    t0 = time.perf_counter()
    O.place(*inputs[0])
    single = C_PER_SCEN * N_PER_SCEN / (time.perf_counter() - t0)

    def one(s):
        cont, nodes = inputs[s % threads] if s < threads else O.gen_scenario(SEED, s, C_PER_SCEN, N_PER_SCEN, FLAGS)
        O.place(cont, nodes)

    done = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < budget_s and done < S_LOCAL:
            n = min(threads, S_LOCAL - done)
            list(ex.map(one, range(done, done + n)))
            done += n
    wall = time.perf_counter() - t0
    return {"value": done * C_PER_SCEN * N_PER_SCEN / wall, "unit": "evals/s", "cores": threads, "kind": "port",
            "single_thread_value": single,
            "sample": f"{done} whole scenarios of 50k x 5k, {threads} at a time on {threads} host threads "
                      f"(oracle/fp_oracle.c fpo_place: sort + first-fit scan), {wall:.1f} s wall"}


def load_traffic():
    """HBM bytes per FFD launch from the committed rocprofv3 --pmc summary, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_ffd_latest.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("scenarios_per_launch") == S_LOCAL and d.get("C") == C_PER_SCEN and d.get("N") == N_PER_SCEN:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from fleetflow_amd import DevBatch, Planner, shard
    from fleetflow_amd._lib import FP_K_PLACE, FP_K_SORT

    S = args.scenarios_per_gpu
    C, N = C_PER_SCEN, N_PER_SCEN
    planner = Planner(local_rank)
    # one dedicated stream for torch's copies/collectives AND the planner kernels
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    planner.set_stream(stream.cuda_stream)
    base, _ = shard.block(rank, world, S * world)
    db = DevBatch.allocate(S, C, N, dev, scen_base=base)
    planner.dev_gen_batch(SEED, db, FLAGS)
    pristine = db.node_snapshot()
    best = torch.empty(1, dtype=torch.int32, device=dev)

    def step():
        db.restore_nodes(pristine)
        planner.dev_place_batch(db)
        if world > 1:
            planner.dev_argmin_cost(shard.gather_costs(db.cost, world, S * world), best)
        else:
            planner.dev_argmin_cost(db.cost, best)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    ref_cost = db.cost.clone()
    ref_assign_sum = int(db.assign.sum().item())
    planner.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    # every timed step re-planned the same inputs: its plans must be bit-identical
    if not torch.equal(db.cost, ref_cost) or int(db.assign.sum().item()) != ref_assign_sum:
        raise RuntimeError("timed steps did not reproduce the warmup plan (stream ordering bug?)")
    place_ms, place_n = planner.kernel_stats(FP_K_PLACE)
    sort_ms, sort_n = planner.kernel_stats(FP_K_SORT)
    best_id = int(best.item())

    if rank == 0:
        evals_total = S * world * C * N
        step_s = elapsed / args.steps
        kernel_s = (place_ms / max(place_n, 1)) / 1e3
        evals_launch = S * C * N
        achieved = evals_launch * 16 / kernel_s / 1e9
        traffic = load_traffic()
        out = {
            "metric": "container x node evaluations/sec (FFD what-if plans, work-equivalent) "
                      "+ achieved GB/s % HBM roofline",
            "value": evals_total / step_s,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_s * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SPEC.md 3, SplitMix64 seed 0x5EED0004, generated on device)",
            "config": {"workload": "BASELINE config 4: what-if FFD, 512 scenarios/GPU x 50k containers x 5k "
                                   "nodes, ports+anti-affinity+labels, RCCL all-gather of packed costs + argmin",
                       "scenarios_per_gpu": S, "scenarios_total": S * world, "containers": C, "nodes": N,
                       "parallelism": f"scenario-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                         "traffic_GBps": (traffic / kernel_s / 1e9) if traffic else None,
                         "kernel": "k_ffd_pipe (fp_pipe.hip)", "kernel_ms": kernel_s * 1e3,
                         "units_per_launch": evals_launch, "bytes_per_unit": 16},
            "breakdown_ms": {"ffd_kernel": place_ms / max(place_n, 1), "sort": sort_ms / max(sort_n, 1)},
            "best_scenario": best_id,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_budget_s, args.cpu_threads)
        print(json.dumps(out), flush=True)
    planner.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
