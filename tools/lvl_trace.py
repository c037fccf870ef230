"""Where config 5's levelizer time goes: the first time k_lvl_async wrote each level, from the
diagnostics build (FP_LVL_TRACE; make -C fleetflow_amd/csrc BUILD=build/lvltrace
OUT=../libfleetplace_lvltrace.so EXTRA=-DFP_LVL_TRACE).
    FLEETPLACE_LIB=.../libfleetplace_lvltrace.so python tools/lvl_trace.py [dag=c,l,L,w,y] [option=value ...]
(dag: chains, chain length, layers, layer width, 3-cycles; default bench.py's config 5)
Prints one JSON line per call: the kernel span, the time to the first level, the chain part
(levels 1..499 of the 500-long chains: us per level), the join part above it, and the drain
after the last level (termination)."""
import ctypes as ct
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from fleetflow_amd import Planner, _lib, synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    args = [a for a in sys.argv[1:] if not a.startswith("dag=")]
    dag = [tuple(int(x) for x in a[4:].split(",")) for a in sys.argv[1:] if a.startswith("dag=")]
    dag = dag[0] if dag else bench.DAG5
    rp, col, hd = synth.gen_dag(bench.SEED5, *dag)
    V = hd.size
    to = lambda a: torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).to(dev)  # noqa: E731
    rp_t, col_t, hd_t = to(rp), to(col), to(hd)
    level_t = torch.empty(V, dtype=torch.int32, device=dev)
    order_t = torch.empty(V, dtype=torch.int32, device=dev)
    ncyc_t = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = ct.CDLL(_lib.LIB_PATH)
    f = lib.fp_debug_lvl_trace
    f.argtypes = [ct.c_void_p]
    buf = np.zeros(4096, np.uint64)
    chain = dag[1]
    with Planner(0) as p:
        for kv in args:
            k, v = kv.split("=")
            p.set_option(k, int(v))
        for call in range(4):
            p.dev_levelize(rp_t, col_t, hd_t, level_t, order_t, ncyc_t)
            p.sync()
            assert f(buf.ctypes.data) == 0
            t0, t1 = int(buf[4094]), int(buf[4095])
            lv = buf[:4094]
            seen = np.nonzero(lv != np.uint64(0xFFFFFFFFFFFFFFFF))[0]
            top = int(seen.max())
            us = lambda t: (int(t) - t0) / 100.0  # noqa: E731  (100 MHz)
            unset = np.uint64(0xFFFFFFFFFFFFFFFF)
            rel = np.array([us(lv[L]) if lv[L] != unset else np.nan for L in range(top + 1)])
            c_end = max(min(chain - 1, top), 1)
            out = {"call": call, "span_us": us(t1), "first_level_us": round(rel[1], 2),
                   "chain_end_level": c_end, "chain_end_us": round(rel[c_end], 2),
                   "chain_us_per_level": round((rel[c_end] - rel[1]) / max(c_end - 1, 1), 3),
                   "top_level": top, "top_us": round(rel[top], 2),
                   "join_us_per_level": round((rel[top] - rel[c_end]) / max(top - c_end, 1), 2),
                   "drain_us": round(us(t1) - rel[top], 2),
                   "dag": list(dag),
                   "recorded": [[int(L), round(float(rel[L]), 2)] for L in range(top + 1) if not np.isnan(rel[L])][:60],
                   "levels_us": {str(L): round(rel[L], 2) for L in
                                 sorted(set(list(range(1, c_end, 50)) + list(range(c_end, top + 1))))}}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
