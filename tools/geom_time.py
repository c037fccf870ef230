"""Time fp_dev_place_batch at 512 x 50k with N = 3000 / 1500 nodes (10-group and fewer-group stages)."""
import os, sys, time, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import DevBatch, Planner, _lib
for N in (3000, 1500):
    S, C = 512, 50000
    p = Planner(0)
    _opts.apply_env(p)
    db = DevBatch.allocate(S, C, N, "cuda:0")
    p.dev_gen_batch(0x5EED0004, db, 7)
    p.sync()
    snap = db.node_snapshot()
    p.profile(True)
    ts = []
    for r in range(4):
        db.restore_nodes(snap); torch.cuda.synchronize()
        t0 = time.perf_counter(); p.dev_place_batch(db); p.sync(); ts.append(time.perf_counter() - t0)
    ms, n = p.kernel_stats(_lib.FP_K_PLACE)
    print(json.dumps({"lib": os.path.basename(os.environ.get("FLEETPLACE_LIB", "default")), "N": N, "wall_ms": round(min(ts[1:]) * 1e3, 3), "kernel_ms": round(ms / n, 3), "cost0": int(db.cost[0].item())}), flush=True)
