"""Diagnostics: systolic group-fill calls on one workload (stats build): calls, queued containers,
live nodes, steps, placements, live nodes some queued container fits, last placement position.

    tools/build_variant.sh _statsfine -DFP_PIPE_STATS -DFP_PIPE_STATS_FINE
    FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_statsfine.so python tools/sys_stats.py [S C N seed]
"""
import ctypes as ct
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FLEETPLACE_LIB", os.path.join(ROOT, "fleetflow_amd", "libfleetplace_stats.so"))

import torch  # noqa: E402

from fleetflow_amd import DevBatch, Planner, _lib  # noqa: E402


def main():
    a = sys.argv[1:]
    S, C, N = (int(a[0]), int(a[1]), int(a[2])) if len(a) >= 3 else (1, 1_000_000, 100_000)
    seed = int(a[3], 0) if len(a) >= 4 else 0x5EED0003
    with Planner(0) as p:
        db = DevBatch.allocate(S, C, N, "cuda:0")
        p.dev_gen_batch(seed, db, 7)
        p.sync()
        torch.cuda.synchronize()
        f = _lib.load().fp_debug_sys_stats
        f.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
        buf = (ct.c_ulonglong * 8)()
        f(buf, 1)
        p.dev_place_batch(db)
        p.sync()
        f(buf, 1)
        n = max(buf[0], 1)
        keys = ("calls", "queued", "live", "steps", "placed", "live_useful", "last_pos_plus1")
        out = {k: buf[i] for i, k in enumerate(keys)}
        out.update({"per_call": {k: buf[i] / n for i, k in enumerate(keys) if i},
                    "steps_per_placement": buf[3] / max(buf[4], 1), "S": S, "C": C, "N": N})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
