"""ctypes/numpy wrapper of the C oracle (oracle/libfporacle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and the
cpu_baseline leg of bench.py -- never by the product package.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libfporacle.so")
_lib = None

NONE = 0xFFFFFFFF

u8p = ct.POINTER(ct.c_uint8)
u32p = ct.POINTER(ct.c_uint32)
u64p = ct.POINTER(ct.c_uint64)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ct.CDLL(_SO)
        L.fpo_legacy_order.argtypes = [ct.c_uint32, u8p, u32p]
        L.fpo_levelize.argtypes = [ct.c_uint32, u32p, u32p, u8p, u32p, u32p]
        L.fpo_levelize.restype = ct.c_uint32
        L.fpo_ffd_order.argtypes = [ct.c_uint32, u32p, u32p, u32p]
        L.fpo_place.argtypes = [ct.c_uint32, u32p, u32p, u32p, u32p, ct.c_uint32, u32p, u32p, u32p,
                                u32p, u8p, u32p, u32p, u8p, u64p]
        L.fpo_place.restype = ct.c_uint32
        L.fpo_feasibility.argtypes = [ct.c_uint32, u32p, u32p, u32p, u32p, ct.c_uint32, u32p, u32p,
                                      u32p, u32p, u8p, u32p, u32p, u64p]
        L.fpo_cost.argtypes = [ct.c_uint32, u32p, ct.c_uint32, ct.c_uint32]
        L.fpo_cost.restype = ct.c_uint64
        L.fpo_splitmix_draw.argtypes = [ct.c_uint64, ct.c_uint64]
        L.fpo_splitmix_draw.restype = ct.c_uint64
        L.fpo_scenario_seed.argtypes = [ct.c_uint64, ct.c_uint32]
        L.fpo_scenario_seed.restype = ct.c_uint64
        L.fpo_gen_containers.argtypes = [ct.c_uint64, ct.c_uint32, ct.c_uint32, u32p, u32p, u32p, u32p]
        L.fpo_gen_nodes.argtypes = [ct.c_uint64, ct.c_uint32, ct.c_uint32, u32p, u32p, u32p, u32p, u8p]
        L.fpo_gen_dag.argtypes = [ct.c_uint64, ct.c_uint32, ct.c_uint32, ct.c_uint32, ct.c_uint32,
                                  ct.c_uint32, u32p, u32p, u8p]
        L.fpo_gen_dag.restype = ct.c_uint32
        L.fpo_dag_vertices.argtypes = [ct.c_uint32] * 4
        L.fpo_dag_vertices.restype = ct.c_uint32
        _lib = L
    return _lib


def _p(a, t):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(t)


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _u8(a):
    return np.ascontiguousarray(a, dtype=np.uint8)


def legacy_order(has_deps):
    hd = _u8(has_deps)
    out = np.empty(hd.size, np.uint32)
    lib().fpo_legacy_order(hd.size, _p(hd, u8p), _p(out, u32p))
    return out


def levelize(row_ptr, col, has_deps):
    rp, cl, hd = _u32(row_ptr), _u32(col), _u8(has_deps)
    V = hd.size
    level = np.empty(V, np.uint32)
    order = np.empty(V, np.uint32)
    ncyc = lib().fpo_levelize(V, _p(rp, u32p), _p(cl, u32p), _p(hd, u8p), _p(level, u32p), _p(order, u32p))
    return level, order, int(ncyc)


def ffd_order(cpu, mem):
    c, m = _u32(cpu), _u32(mem)
    out = np.empty(c.size, np.uint32)
    lib().fpo_ffd_order(c.size, _p(c, u32p), _p(m, u32p), _p(out, u32p))
    return out


def place(cont, nodes, level=None, count_evals=False):
    """cont = (cpu, mem, req, conf); nodes = (cf, mf, lab, cu, sched) -- copied, not mutated.
    Returns (assign, reason, nodes_after, evals)."""
    cpu, mem, req, conf = (_u32(x) for x in cont)
    cf, mf, lab, cu = (_u32(x).copy() for x in nodes[:4])
    sched = _u8(nodes[4])
    C, N = cpu.size, cf.size
    assign = np.empty(C, np.uint32)
    reason = np.empty(C, np.uint8)
    lv = _u32(level) if level is not None else None
    ev = ct.c_uint64(0)
    lib().fpo_place(C, _p(cpu, u32p), _p(mem, u32p), _p(req, u32p), _p(conf, u32p), N, _p(cf, u32p),
                    _p(mf, u32p), _p(lab, u32p), _p(cu, u32p), _p(sched, u8p), _p(lv, u32p),
                    _p(assign, u32p), _p(reason, u8p), ct.byref(ev) if count_evals else None)
    return assign, reason, (cf, mf, lab, cu, sched), int(ev.value)


def feasibility(cont, nodes, want_bitmap=True):
    cpu, mem, req, conf = (_u32(x) for x in cont)
    cf, mf, lab, cu = (_u32(x) for x in nodes[:4])
    sched = _u8(nodes[4])
    C, N = cpu.size, cf.size
    first = np.empty(C, np.uint32)
    count = np.empty(C, np.uint32)
    bm = np.zeros(((C + 63) // 64) * N, np.uint64) if want_bitmap else None
    lib().fpo_feasibility(C, _p(cpu, u32p), _p(mem, u32p), _p(req, u32p), _p(conf, u32p), N, _p(cf, u32p),
                          _p(mf, u32p), _p(lab, u32p), _p(cu, u32p), _p(sched, u8p), _p(first, u32p),
                          _p(count, u32p), _p(bm, u64p))
    return first, count, bm


def cost(assign, n_nodes, scenario_id):
    a = _u32(assign)
    return int(lib().fpo_cost(a.size, _p(a, u32p), n_nodes, scenario_id))


def scenario_seed(seed, s):
    return int(lib().fpo_scenario_seed(seed, s))


def gen_containers(seed, C, flags):
    out = [np.empty(C, np.uint32) for _ in range(4)]
    lib().fpo_gen_containers(seed, C, flags, *(_p(o, u32p) for o in out))
    return tuple(out)


def gen_nodes(seed, N, flags=7):
    cf, mf, lab, cu = (np.empty(N, np.uint32) for _ in range(4))
    sched = np.empty(N, np.uint8)
    lib().fpo_gen_nodes(seed, N, flags, _p(cf, u32p), _p(mf, u32p), _p(lab, u32p), _p(cu, u32p), _p(sched, u8p))
    return cf, mf, lab, cu, sched


def gen_scenario(seed, scenario, C, N, flags):
    s = scenario_seed(seed, scenario)
    return gen_containers(s, C, flags), gen_nodes(s, N, flags)


def gen_dag(seed, n_chains, chain_len, n_layers, layer_width, n_cycles):
    L = lib()
    V = L.fpo_dag_vertices(n_chains, chain_len, n_layers, layer_width)
    row_ptr = np.empty(V + 1, np.uint32)
    hd = np.empty(V, np.uint8)
    E = L.fpo_gen_dag(seed, n_chains, chain_len, n_layers, layer_width, n_cycles, _p(row_ptr, u32p), None,
                      _p(hd, u8p))
    col = np.empty(max(E, 1), np.uint32)
    L.fpo_gen_dag(seed, n_chains, chain_len, n_layers, layer_width, n_cycles, _p(row_ptr, u32p),
                  _p(col, u32p), _p(hd, u8p))
    return row_ptr, col[:E], hd
