"""Levelization time vs DAG shape (chains only, layers only, both): where the
asynchronous levelizer's time goes.  python tools/lvl_shapes.py"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import Planner  # noqa: E402
from oracle import oracle as O  # noqa: E402  (input generator only)


def run(p, dev, shape):
    rp, col, hd = O.gen_dag(0x5EED0005, *shape)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)  # noqa: E731
    rp_t, col_t, hd_t = t(rp), t(col if col.size else np.zeros(1, np.uint32)), torch.from_numpy(hd).to(dev)
    V = hd.size
    lv = torch.empty(V, dtype=torch.int32, device=dev)
    od = torch.empty(V, dtype=torch.int32, device=dev)
    nc = torch.zeros(1, dtype=torch.int32, device=dev)
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.dev_levelize(rp_t, col_t, hd_t, lv, od, nc)
        p.sync()
        walls.append((time.perf_counter() - t0) * 1e3)
    levels = int(lv.cpu().numpy().view(np.uint32)[lv.cpu().numpy().view(np.uint32) != 0xFFFFFFFF].max()) + 1
    return {"shape": shape, "V": V, "E": int(col.size), "levels": levels, "ms": round(min(walls[1:]), 3),
            "us_per_level": round(min(walls[1:]) * 1e3 / levels, 2)}


def main():
    dev = torch.device("cuda", 0)
    with Planner(0) as p:
        _opts.apply_env(p)
        for shape in [(1000, 500, 0, 0, 0), (1, 500, 0, 0, 0), (1000, 100, 0, 0, 0), (100, 1, 50, 10_000, 0),
                      (1000, 500, 50, 10_000, 333)]:
            print(json.dumps(run(p, dev, shape)), flush=True)


if __name__ == "__main__":
    main()
