"""Config-5 levelization timing (bench.py's levelize_leg, kernel and wall ms) on cuda:0.
    python tools/lvl_time.py [dag=c,l,L,w,y] [option=value ...]   (context options, _lib.OPTIONS names;
    dag: chains, chain length, layers, layer width, 3-cycles -- default bench.py's config 5)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from fleetflow_amd import Planner  # noqa: E402

dag = [tuple(int(x) for x in a[4:].split(",")) for a in sys.argv[1:] if a.startswith("dag=")]
if dag:
    bench.DAG5 = dag[0]
with Planner(0) as p:
    for kv in sys.argv[1:]:
        k, v = kv.split("=")
        if k != "dag":
            p.set_option(k, int(v))
    for _ in range(2):
        lv = bench.levelize_leg(p, torch.device("cuda", 0), 10)[0]
        print(json.dumps({k: lv[k] for k in ("ms_per_step", "kernel_ms", "levels", "cycle_vertices")}), flush=True)
