"""Diagnostics: config-4 FFD kernel time (HIP events, fp_ctx_kernel_stats) under the two ways the
tools drive the planner -- (a) tools/sys_sweep.py: the context's own stream, a device sync between
calls; (b) bench.py: a torch stream handed to the context, steps back to back -- and (c) the bench's
stream with a sync between calls.  One JSON line per mode.
    python tools/stream_ab.py [S]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from fleetflow_amd import DevBatch, Planner  # noqa: E402
from fleetflow_amd._lib import FP_K_PLACE  # noqa: E402


def run(p, db, snap, reps, sync_each):
    times = []
    p.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        db.restore_nodes(snap)
        if sync_each:
            torch.cuda.synchronize()
        p.dev_place_batch(db)
        if sync_each:
            p.sync()
            ms, n = p.kernel_stats(FP_K_PLACE)
            times.append(ms / max(n, 1))
            p.profile(False)
            p.profile(True)
    p.sync()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    if not sync_each:
        ms, n = p.kernel_stats(FP_K_PLACE)
        times.append(ms / max(n, 1))
    p.profile(False)
    return statistics.median(times), wall


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda", 0)
    with Planner(0) as p:
        db = DevBatch.allocate(S, 50_000, 5_000, dev)
        p.dev_gen_batch(0x5EED0004, db, 7)
        p.sync()
        snap = db.node_snapshot()
        torch.cuda.synchronize()
        run(p, db, snap, 1, True)
        for mode in ("own_stream_sync", "torch_stream_back_to_back", "torch_stream_sync", "own_stream_sync"):
            if mode.startswith("torch"):
                st = torch.cuda.Stream(dev)
                torch.cuda.set_stream(st)
                p.set_stream(st.cuda_stream)
            else:
                torch.cuda.set_stream(torch.cuda.default_stream(dev))
                p.reset_stream()
            k, w = run(p, db, snap, 5, mode.endswith("sync"))
            print(json.dumps({"mode": mode, "S": S, "ffd_ms": round(k, 3), "wall_ms_per_call": round(w, 3)}), flush=True)


if __name__ == "__main__":
    main()
