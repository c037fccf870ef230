"""Host-side wrappers over the C ABI (include/fleetplace.h).

``Planner`` owns one ``fp_ctx`` (one HIP stream on one MI355X).  The numpy
methods use the synchronous host-pointer entry points (the drop-in boundary a
Rust/cgo caller would use); ``DevBatch`` + the ``dev_*`` methods run the same
kernels on device-resident tensors (torch is only the HBM allocator here).
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import FpBatch, FpContainers, FpGraph, FpNodes, check

NONE = _lib.FP_NONE


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _u8(a):
    return np.ascontiguousarray(a, dtype=np.uint8)


def _ptr(a):
    return None if a is None else a.ctypes.data


class Planner:
    def __init__(self, device: int = 0):
        self._L = _lib.load()
        h = ct.c_void_p()
        check(self._L.fp_ctx_create(ct.byref(h), device), "fp_ctx_create")
        self._ctx = h
        self.device = device
        self._tstream = None  # torch view of the stream the dev_* calls launch on (see _dev)

    # -- lifetime ---------------------------------------------------------------
    def close(self):
        if getattr(self, "_ctx", None):
            if getattr(self, "_tstream", None) is not None:
                self._L.fp_ctx_reset_stream(self._ctx)  # off the torch stream before it can go away
                self._tstream = None
            self._L.fp_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_stream(self, hip_stream_handle: int):
        """Launch on this hipStream_t handle; 0 is the HIP null (default) stream."""
        check(self._L.fp_ctx_set_stream(self._ctx, ct.c_void_p(int(hip_stream_handle))), "fp_ctx_set_stream")
        import torch
        self._tstream = torch.cuda.ExternalStream(int(hip_stream_handle), device=torch.device("cuda", self.device))

    def reset_stream(self):
        check(self._L.fp_ctx_reset_stream(self._ctx), "fp_ctx_reset_stream")
        self._tstream = None

    def _dev(self, fn, *args):
        """Run one fp_dev_* call ordered with torch's current stream on both sides: the call
        waits for work queued there before it (a restore_nodes copy, a tensor fill) and later
        work there waits for the call (a snapshot, a comparison).  Stream-ordered, no host
        sync.  The context launches on a torch-created stream unless set_stream chose one."""
        import torch
        cur = torch.cuda.current_stream(self.device)
        if self._tstream is None:
            st = torch.cuda.Stream(device=torch.device("cuda", self.device))
            check(self._L.fp_ctx_set_stream(self._ctx, ct.c_void_p(st.cuda_stream)), "fp_ctx_set_stream")
            self._tstream = st
        if self._tstream.cuda_stream == cur.cuda_stream:
            return fn(*args)
        self._tstream.wait_stream(cur)
        try:
            return fn(*args)
        finally:
            cur.wait_stream(self._tstream)

    def sync(self):
        check(self._L.fp_ctx_sync(self._ctx), "fp_ctx_sync")

    def profile(self, enable=True):
        check(self._L.fp_ctx_profile(self._ctx, int(enable)), "fp_ctx_profile")

    def set_option(self, name: str, value: int = _lib.FP_OPT_AUTO):
        """fp_ctx_set_option by name (_lib.OPTIONS); FP_OPT_AUTO (-1) restores the default."""
        check(self._L.fp_ctx_set_option(self._ctx, _lib.OPTIONS[name], int(value)), f"fp_ctx_set_option({name})")

    def get_option(self, name: str) -> int:
        v = ct.c_int64()
        check(self._L.fp_ctx_get_option(self._ctx, _lib.OPTIONS[name], ct.byref(v)), f"fp_ctx_get_option({name})")
        return int(v.value)

    def reset_options(self):
        for name in _lib.OPTIONS:
            self.set_option(name, _lib.FP_OPT_AUTO)

    def geometry(self, S: int, C: int, N: int) -> dict:
        """The placement pipeline a batch of S x C x N runs on this context (fp_place_geometry)."""
        out = (ct.c_uint32 * len(_lib.GEOM_FIELDS))()
        check(self._L.fp_place_geometry(self._ctx, S, C, N, out), "fp_place_geometry")
        return dict(zip(_lib.GEOM_FIELDS, (int(x) for x in out)))

    def place_path(self) -> dict:
        """The FFD kernel the last placement ran (fp_ctx_place_path; waits for the stream):
        {"or_cpu", "or_mem", "packed"} -- packed is True for the packed (cpu, mem) records."""
        out = (ct.c_uint32 * 3)()
        check(self._L.fp_ctx_place_path(self._ctx, out), "fp_ctx_place_path")
        return {"or_cpu": int(out[0]), "or_mem": int(out[1]), "packed": int(out[2]) == 2, "ran": int(out[2]) != 0}

    def kernel_stats(self, kernel_id: int):
        ms = ct.c_double()
        n = ct.c_uint64()
        check(self._L.fp_ctx_kernel_stats(self._ctx, kernel_id, ct.byref(ms), ct.byref(n)), "kernel_stats")
        return ms.value, n.value

    # -- host-pointer API ------------------------------------------------------------
    # Every array is read (or written) for the length the call's sizes imply, so a shorter one would be
    # read out of bounds by the library: refused with ValueError first, as lib.rs returns FP_EINVAL.
    @staticmethod
    def _need(cond, what):
        if not cond:
            raise ValueError(what)

    def legacy_order(self, has_deps):
        """engine.rs:67-85 on indices: has_deps[i] = known && depends_on non-empty."""
        hd = _u8(has_deps)
        out = np.empty(hd.size, np.uint32)
        g = FpGraph(hd.size, 0, None, None, _ptr(hd))
        check(self._L.fp_legacy_order(self._ctx, ct.byref(g), out.ctypes.data_as(_lib.u32p)), "fp_legacy_order")
        return out

    def levelize(self, row_ptr, col, has_deps):
        rp, cl, hd = _u32(row_ptr), _u32(col), _u8(has_deps)
        V = hd.size
        self._need(V == 0 or rp.size == V + 1, "row_ptr must hold V + 1 entries")
        level = np.empty(V, np.uint32)
        order = np.empty(V, np.uint32)
        ncyc = ct.c_uint32()
        g = FpGraph(V, cl.size, _ptr(rp), _ptr(cl) if cl.size else None, _ptr(hd))
        check(self._L.fp_levelize(self._ctx, ct.byref(g), level.ctypes.data_as(_lib.u32p),
                                  order.ctypes.data_as(_lib.u32p), ct.byref(ncyc)), "fp_levelize")
        return level, order, ncyc.value

    def plan_stage_lists(self, row_ptr, col, has_deps):
        """fp_plan_stage without servers for a graph given as Python sequences (a fleet.kdl stage;
        BASELINE config 1 is timed per plan, where numpy conversions and ctypes argument conversion
        cost more than the GPU work): the inputs go into ctypes buffers kept between calls, the call
        is one prebuilt foreign call, and the results come back as lists.  Returns (perm, level,
        order, n_cycle).  Same checks and errors as plan_stage."""
        V, E = len(has_deps), len(col)
        self._need(V == 0 or len(row_ptr) == V + 1, "row_ptr must hold V + 1 entries")
        fs = getattr(self, "_fs", None)
        if fs is None or V > fs["V"] or E > fs["E"]:
            cv, ce = max(64, V), max(256, E)
            rp, cl, hd = (ct.c_uint32 * (cv + 1))(), (ct.c_uint32 * ce)(), (ct.c_uint8 * cv)()
            out, ncyc = (ct.c_uint32 * (3 * cv))(), ct.c_uint32()
            g = FpGraph(0, 0, ct.addressof(rp), ct.addressof(cl), ct.addressof(hd))
            a = ct.addressof(out)
            args = (self._ctx, ct.byref(g), None, None, ct.c_void_p(a), ct.c_void_p(a + 4 * cv),
                    ct.c_void_p(a + 8 * cv), ct.byref(ncyc), None, None, None, None)
            fs = self._fs = {"V": cv, "E": ce, "rp": rp, "col": cl, "hd": hd, "out": out, "ncyc": ncyc, "g": g,
                             "args": args, "fn": _lib.raw_function("fp_plan_stage")}
        if V == 0:
            return [], [], [], 0
        fs["rp"][:V + 1] = row_ptr
        if E:
            fs["col"][:E] = col
        fs["hd"][:V] = has_deps
        g = fs["g"]
        g.n_vertices = V
        g.n_edges = E
        check(fs["fn"](*fs["args"]), "fp_plan_stage")
        out, cv = fs["out"], fs["V"]
        return out[:V], out[cv:cv + V], out[2 * cv:2 * cv + V], fs["ncyc"].value

    def plan_stage(self, row_ptr, col, has_deps, cont=None, nodes=None):
        """fp_plan_stage: one stage's A1 legacy order, A2 levels and start order and, with ``nodes``
        (container v = vertex v), the stage-2 candidates on the pristine table and the FFD plan gated
        by the levels' CYCLE -- one call (one kernel for a fleet.kdl-sized stage).  Returns
        (perm, level, order, n_cycle, placed) with placed = None or (first, count, assign, reason,
        nodes_after)."""
        rp, cl, hd = _u32(row_ptr), _u32(col), _u8(has_deps)
        V = hd.size
        self._need(V == 0 or rp.size == V + 1, "row_ptr must hold V + 1 entries")
        out = np.empty(3 * V, np.uint32)  # perm, level, order: one allocation, passed as addresses
        perm, level, order = out[:V], out[V:2 * V], out[2 * V:]
        o = out.ctypes.data
        ncyc = ct.c_uint32()
        g = FpGraph(V, cl.size, rp.ctypes.data, cl.ctypes.data if cl.size else None, hd.ctypes.data)
        if nodes is None:
            check(self._L.fp_plan_stage(self._ctx, ct.byref(g), None, None, o, o + 4 * V, o + 8 * V, ct.byref(ncyc),
                                        None, None, None, None), "fp_plan_stage")
            return perm, level, order, ncyc.value, None
        cpu, mem, req, conf = (_u32(x) for x in cont)
        cf, mf = _u32(nodes[0]).copy(), _u32(nodes[1]).copy()
        lab, cu, sched = _u32(nodes[2]), _u32(nodes[3]).copy(), _u8(nodes[4])
        self._need(all(x.size == V for x in (cpu, mem, req, conf)), "every container array must hold V entries")
        self._need(all(x.size == cf.size for x in (mf, lab, cu, sched)), "every node array must hold N entries")
        first = np.empty(V, np.uint32)
        count = np.empty(V, np.uint32)
        assign = np.empty(V, np.uint32)
        reason = np.empty(V, np.uint8)
        cs = FpContainers(V, _ptr(cpu), _ptr(mem), _ptr(req), _ptr(conf))
        ns = FpNodes(cf.size, _ptr(cf), _ptr(mf), _ptr(lab), _ptr(cu), _ptr(sched))
        check(self._L.fp_plan_stage(self._ctx, ct.byref(g), ct.byref(cs), ct.byref(ns), o, o + 4 * V, o + 8 * V,
                                    ct.byref(ncyc), first.ctypes.data, count.ctypes.data, assign.ctypes.data,
                                    reason.ctypes.data), "fp_plan_stage")
        return perm, level, order, ncyc.value, (first, count, assign, reason, (cf, mf, lab, cu, sched))

    def place(self, cont, nodes, level=None):
        """cont = (cpu_m, mem_mib, req_labels, conflict); nodes = (cpu_free, mem_free,
        labels, conflict_used, schedulable).  Inputs are not mutated; the updated node
        state is returned.  Returns (assign, reason, nodes_after)."""
        cpu, mem, req, conf = (_u32(x) for x in cont)
        cf, mf = _u32(nodes[0]).copy(), _u32(nodes[1]).copy()
        lab, cu, sched = _u32(nodes[2]), _u32(nodes[3]).copy(), _u8(nodes[4])
        C, N = cpu.size, cf.size
        lv = _u32(level) if level is not None else None
        self._need(all(x.size == C for x in (mem, req, conf)), "every container array must hold C entries")
        self._need(all(x.size == N for x in (mf, lab, cu, sched)), "every node array must hold N entries")
        self._need(lv is None or lv.size == C, "level must hold C entries")
        assign = np.empty(C, np.uint32)
        reason = np.empty(C, np.uint8)
        cs = FpContainers(C, _ptr(cpu), _ptr(mem), _ptr(req), _ptr(conf))
        ns = FpNodes(N, _ptr(cf), _ptr(mf), _ptr(lab), _ptr(cu), _ptr(sched))
        check(self._L.fp_place(self._ctx, ct.byref(cs), ct.byref(ns),
                               lv.ctypes.data_as(_lib.u32p) if lv is not None else None,
                               assign.ctypes.data_as(_lib.u32p), reason.ctypes.data_as(_lib.u8p)), "fp_place")
        return assign, reason, (cf, mf, lab, cu, sched)

    def place_batch(self, S, C, N, cont, nodes, level=None, scen_base=0):
        """Scenario-major arrays ([S*C] containers, [S*N] nodes).  Returns
        (assign, reason, cost, nodes_after)."""
        cpu, mem, req, conf = (_u32(x) for x in cont)
        cf, mf = _u32(nodes[0]).copy(), _u32(nodes[1]).copy()
        lab, cu, sched = _u32(nodes[2]), _u32(nodes[3]).copy(), _u8(nodes[4])
        lv = _u32(level) if level is not None else None
        self._need(all(x.size == S * C for x in (cpu, mem, req, conf)), "every container array must hold S * C entries")
        self._need(all(x.size == S * N for x in (cf, mf, lab, cu, sched)), "every node array must hold S * N entries")
        self._need(lv is None or lv.size == S * C, "level must hold S * C entries")
        assign = np.empty(S * C, np.uint32)
        reason = np.empty(S * C, np.uint8)
        cost = np.empty(S, np.uint64)
        b = FpBatch(S, scen_base, C, N, _ptr(cpu), _ptr(mem), _ptr(req), _ptr(conf), _ptr(lv), _ptr(cf),
                    _ptr(mf), _ptr(lab), _ptr(cu), _ptr(sched), _ptr(assign), _ptr(reason), _ptr(cost))
        check(self._L.fp_place_batch(self._ctx, ct.byref(b)), "fp_place_batch")
        return assign, reason, cost, (cf, mf, lab, cu, sched)

    def feasibility(self, cont, nodes, bitmap=True):
        cpu, mem, req, conf = (_u32(x) for x in cont)
        cf, mf, lab, cu = (_u32(x) for x in nodes[:4])
        sched = _u8(nodes[4])
        C, N = cpu.size, cf.size
        first = np.empty(C, np.uint32)
        count = np.empty(C, np.uint32)
        bm = np.empty(((C + 63) // 64) * N, np.uint64) if bitmap else None
        cs = FpContainers(C, _ptr(cpu), _ptr(mem), _ptr(req), _ptr(conf))
        ns = FpNodes(N, _ptr(cf), _ptr(mf), _ptr(lab), _ptr(cu), _ptr(sched))
        check(self._L.fp_feasibility(self._ctx, ct.byref(cs), ct.byref(ns), first.ctypes.data_as(_lib.u32p),
                                     count.ctypes.data_as(_lib.u32p),
                                     bm.ctypes.data_as(_lib.u64p) if bm is not None else None), "fp_feasibility")
        return first, count, bm

    # -- device-pointer API -------------------------------------------------------------
    def dev_gen_batch(self, seed, db: "DevBatch", flags=7):
        self._dev(lambda: check(self._L.fp_dev_gen_batch(self._ctx, ct.c_uint64(seed), ct.byref(db.struct()), flags),
                                "fp_dev_gen_batch"))

    def dev_place_batch(self, db: "DevBatch"):
        self._dev(lambda: check(self._L.fp_dev_place_batch(self._ctx, ct.byref(db.struct())), "fp_dev_place_batch"))

    def dev_argmin_cost(self, cost_t, out_t):
        self._dev(lambda: check(self._L.fp_dev_argmin_cost(self._ctx, cost_t.data_ptr(), cost_t.numel(),
                                                           out_t.data_ptr()), "fp_dev_argmin_cost"))

    def dev_feasibility(self, db: "DevBatch", first_t, count_t, bitmap_t=None, scenario=0):
        C, N = db.C, db.N
        o, p = scenario * C, scenario * N
        cs = FpContainers(C, db.cpu[o:].data_ptr(), db.mem[o:].data_ptr(), db.req[o:].data_ptr(),
                          db.conf[o:].data_ptr())
        ns = FpNodes(N, db.cf[p:].data_ptr(), db.mf[p:].data_ptr(), db.lab[p:].data_ptr(), db.cu[p:].data_ptr(),
                     db.sched[p:].data_ptr())
        self._dev(lambda: check(self._L.fp_dev_feasibility(
            self._ctx, ct.byref(cs), ct.byref(ns), first_t.data_ptr(), count_t.data_ptr(),
            bitmap_t.data_ptr() if bitmap_t is not None else None), "fp_dev_feasibility"))

    def place_ws_bytes(self, S: int, C: int, N: int) -> int:
        """Device workspace bytes a place batch of S x C x N takes on this context."""
        out = ct.c_uint64(0)
        check(self._L.fp_place_ws_bytes(self._ctx, S, C, N, ct.byref(out)), "fp_place_ws_bytes")
        return int(out.value)

    def dev_feasibility_batch(self, db: "DevBatch", first_t, count_t):
        """Stage 2 over every scenario of ``db`` ([S*C] outputs, scenario-major)."""
        self._dev(lambda: check(self._L.fp_dev_feasibility_batch(self._ctx, ct.byref(db.struct()), first_t.data_ptr(),
                                                                 count_t.data_ptr()), "fp_dev_feasibility_batch"))

    def dev_legacy_order(self, has_deps_t, perm_t):
        """fp_dev_legacy_order (engine.rs:67-85) on a device-resident has_deps vector."""
        g = FpGraph(has_deps_t.numel(), 0, None, None, has_deps_t.data_ptr())
        self._dev(lambda: check(self._L.fp_dev_legacy_order(self._ctx, ct.byref(g), perm_t.data_ptr()),
                                "fp_dev_legacy_order"))

    def dev_levelize(self, row_ptr_t, col_t, has_deps_t, level_t, order_t, ncyc_t):
        V = has_deps_t.numel()
        g = FpGraph(V, col_t.numel(), row_ptr_t.data_ptr(), col_t.data_ptr() if col_t.numel() else None,
                    has_deps_t.data_ptr())
        self._dev(lambda: check(self._L.fp_dev_levelize(self._ctx, ct.byref(g), level_t.data_ptr(), order_t.data_ptr(),
                                                        ncyc_t.data_ptr()), "fp_dev_levelize"))


@dataclass
class DevBatch:
    """Device-resident scenario batch (torch tensors on one GPU, int32 storage
    reinterpreted as uint32 by the kernels)."""
    S: int
    C: int
    N: int
    scen_base: int
    cpu: object
    mem: object
    req: object
    conf: object
    level: object
    cf: object
    mf: object
    lab: object
    cu: object
    sched: object
    assign: object
    reason: object
    cost: object

    @classmethod
    def allocate(cls, S, C, N, device, scen_base=0, with_level=False):
        import torch

        def i32(n):
            return torch.empty(n, dtype=torch.int32, device=device)

        return cls(S, C, N, scen_base, i32(S * C), i32(S * C), i32(S * C), i32(S * C),
                   i32(S * C) if with_level else None, i32(S * N), i32(S * N), i32(S * N), i32(S * N),
                   torch.empty(S * N, dtype=torch.uint8, device=device), i32(S * C),
                   torch.empty(S * C, dtype=torch.uint8, device=device),
                   torch.empty(S, dtype=torch.int64, device=device))

    def struct(self):
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        return FpBatch(self.S, self.scen_base, self.C, self.N, p(self.cpu), p(self.mem), p(self.req),
                       p(self.conf), p(self.level), p(self.cf), p(self.mf), p(self.lab), p(self.cu),
                       p(self.sched), p(self.assign), p(self.reason), p(self.cost))

    def node_snapshot(self):
        """Copies of the node fields a plan mutates (free cpu, free memory, usage count).
        labels and schedulable are const inputs at the boundary (include/fleetplace.h:99-101),
        so they are neither copied nor restored."""
        return tuple(t.clone() for t in (self.cf, self.mf, self.cu))

    def restore_nodes(self, snap):
        for dst, src in zip((self.cf, self.mf, self.cu), snap):
            dst.copy_(src)
