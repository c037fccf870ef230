"""Diagnostics: per-stage counters of the FFD tile pipeline on the bench workload.

    FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_stats.so python tools/pipe_stats.py [S]
"""
import ctypes as ct
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FLEETPLACE_LIB", os.path.join(ROOT, "fleetflow_amd", "libfleetplace_stats.so"))

import torch  # noqa: E402

import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import DevBatch, Planner, _lib  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    C, N = int(os.environ.get("C", 50000)), int(os.environ.get("N", 5000))
    p = Planner(0)
    _opts.apply_env(p)
    db = DevBatch.allocate(S, C, N, "cuda:0")
    p.dev_gen_batch(int(os.environ.get("SEED", "0x5EED0004"), 0), db, 7)
    p.sync()  # the generator runs on the planner stream; torch copies on its own
    pristine = db.node_snapshot()
    torch.cuda.synchronize()
    L = _lib.load()
    f = L.fp_debug_pipe_stats
    f.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
    buf = (ct.c_ulonglong * 256)()
    p.profile(True)
    for rep in range(2):
        db.restore_nodes(pristine)
        torch.cuda.synchronize()
        f(buf, 1)
        t0 = time.perf_counter()
        p.dev_place_batch(db)
        p.sync()
        dt = time.perf_counter() - t0
    ms, n = p.kernel_stats(_lib.FP_K_PLACE)
    f(buf, 0)
    print(f"S={S} C={C} N={N} step {dt*1e3:.2f} ms, ffd kernel avg {ms/n:.2f} ms")
    print("stage  visits/scen  checks/scen  hits/scen  batches/scen  spin_in/batch  spin_out/batch")
    for w in range(16):
        v = [buf[w * 16 + i] for i in range(16)]
        if not any(v):
            continue
        b = max(v[3], 1)
        print(f"{w:5d} {v[0]/S:12.0f} {v[1]/S:12.0f} {v[2]/S:10.0f} {v[3]/S:13.0f} {v[4]/b:14.1f} {v[5]/b:15.1f}")
    print("stage  Mcycles/scen: input  prescan  cand_loop  fwd  out_wait  total   | cycles/check  (checks / mask upkeep / queues / touched: FP_PIPE_STATS_FINE builds)")
    for w in range(16):
        v = [buf[w * 16 + i] for i in range(16)]
        if not any(v):
            continue
        f = lambda x: x / S / 1e6  # noqa: E731
        print(f"{w:5d} {f(v[8]):18.2f} {f(v[9]):8.2f} {f(v[10]):10.2f} {f(v[11]):5.2f} {f(v[12]):9.2f} {f(v[13]):6.2f}"
              f"   | {v[10]/max(v[1],1):8.0f}   in cand_loop: checks {f(v[6]):6.2f} mask upkeep {f(v[7]):6.2f}"
              f"  queues/scen {v[14]/S:7.0f} touched/scen {v[15]/S:7.0f}")




def timeline(out_path):
    """Dump scenario 0's per-batch timeline (stats build) to out_path as CSV (global stage = segment * W + stage):
    s_memtime stamps of the loop top (= the previous batch's end), input available, input read, prescan end and
    group loop end, then checks, hits, todo and the batch's valid containers (tools/front_breakdown.py)."""
    L = _lib.load()
    f = L.fp_debug_pipe_timeline
    f.argtypes = [ct.POINTER(ct.c_ulonglong)]
    TLB = 2048
    buf = (ct.c_ulonglong * (16 * TLB * 8))()
    f(buf)
    with open(out_path, "w") as fo:
        fo.write("stage,batch,t_top,t_avail,t_in,t_pre,t_cand,checks,hits,todo,valid\n")
        for w in range(16):
            for b in range(TLB):
                v = [buf[(w * TLB + b) * 8 + i] for i in range(8)]
                if v[0]:
                    fo.write(f"{w},{b}," + ",".join(str(x) for x in v[:7]) + f",{v[7] & 0xFFFFFFFF},{v[7] >> 32}\n")


def stage_span(out_path):
    """Dump scenario 0's per-stage span (stats build) to out_path as CSV: realtime ticks (100 MHz)."""
    L = _lib.load()
    f = L.fp_debug_stage_span
    f.argtypes = [ct.POINTER(ct.c_ulonglong)]
    buf = (ct.c_ulonglong * (4096 * 8))()
    f(buf)
    with open(out_path, "w") as fo:
        fo.write("stage,start,first,end,busy_cyc,batches,wait_cyc,spin_in,hits\n")
        for w in range(4096):
            v = [buf[w * 8 + i] for i in range(8)]
            if v[0]:
                fo.write(f"{w}," + ",".join(str(x) for x in v) + "\n")


if __name__ == "__main__":
    main()
    if os.environ.get("TIMELINE"):
        timeline(os.environ["TIMELINE"])
    if os.environ.get("SPAN"):
        stage_span(os.environ["SPAN"])
