"""Diagnostics: k_scen_sort phase cycles on the bench workload (stats build).

    python tools/sort_stats.py [S]     (FLEETPLACE_LIB defaults to libfleetplace_stats.so)
"""
import ctypes as ct
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FLEETPLACE_LIB", os.path.join(ROOT, "fleetflow_amd", "libfleetplace_stats.so"))

import torch  # noqa: E402

from fleetflow_amd import DevBatch, Planner, _lib  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    C, N = int(os.environ.get("C", 50000)), int(os.environ.get("N", 5000))
    p = Planner(0)
    db = DevBatch.allocate(S, C, N, "cuda:0")
    p.dev_gen_batch(int(os.environ.get("SEED", "0x5EED0004"), 0), db, 7)
    p.sync()
    pristine = db.node_snapshot()
    torch.cuda.synchronize()
    L = _lib.load()
    f = L.fp_debug_sort_stats
    f.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
    ghz = ct.c_double(0)
    L.fp_debug_clock_ghz.argtypes = [ct.c_void_p, ct.POINTER(ct.c_double)]
    L.fp_debug_clock_ghz(p._ctx, ct.byref(ghz))
    buf = (ct.c_ulonglong * 8)()
    p.profile(True)
    for rep in range(3):
        db.restore_nodes(pristine)
        torch.cuda.synchronize()
        f(buf, 1)
        p.dev_place_batch(db)
        p.sync()
    f(buf, 0)
    sort_ms, n = p.kernel_stats(_lib.FP_K_SORT)
    wg = max(buf[5], 1)
    us = lambda x: x / wg / ghz.value / 1e3  # noqa: E731  per workgroup (scenario), microseconds
    print(f"S={S} C={C} N={N} clock {ghz.value:.3f} GHz, sort path avg {sort_ms / max(n, 1):.3f} ms, workgroups {buf[5]}")
    print(f"per scenario us: R {us(buf[0]):.2f}  A0+offsets {us(buf[1]):.2f}  A1 {us(buf[2]):.2f}  "
          f"B {us(buf[3]):.2f} (busy per wave {us(buf[4]) / 16:.2f})  total {us(buf[7]):.2f}  largest bucket {buf[6]}")
    print(f"resident: 256 CUs x 1 workgroup -> {S / 256:.0f} rounds x {us(buf[7]):.1f} us = "
          f"{S / 256 * us(buf[7]) / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
