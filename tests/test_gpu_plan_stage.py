"""fp_plan_stage: one stage's whole plan in one call (BASELINE config 1).

Every output is checked against the C oracle on the same inputs: the A1 legacy order
(engine.rs:67-85), the A2 levels and start order, the stage-2 candidates on the pristine table
and the FFD plan gated by the levels' CYCLE (SPEC.md 2).  The one-wave path (k_plan_tiny, <= 64
services / 256 edges / 64 servers, inputs in the kernel arguments), the one-workgroup path
(k_plan_small, <= 512 services / 8192 edges / 4096 servers; FP_OPT_LEVEL_SMALL = 2 keeps it for
the tiny shapes too) and the general path (a stage past the limits, or FP_OPT_LEVEL_SMALL = 0) must
agree bit for bit.
"""
import numpy as np
import pytest

from fleetflow_amd.planner import NONE

pytestmark = pytest.mark.gpu


def _csr(V, edges):
    edges = sorted(edges, key=lambda t: t[0])  # stable: per-dep order kept
    rp = np.zeros(V + 1, np.uint32)
    for d, _ in edges:
        rp[d + 1] += 1
    rp = np.cumsum(rp).astype(np.uint32)
    col = np.array([t for _, t in edges], np.uint32)
    return rp, col


def _stage(V, E_extra, seed, cycle=True):
    """A stage-like DAG: a chain, random forward edges, a 3-cycle with a tail and a self loop."""
    rng = np.random.default_rng(seed)
    edges = [(v, v + 1) for v in range(0, V - 8, 3)]
    a, b = rng.integers(0, max(V - 8, 1), E_extra), rng.integers(0, max(V - 8, 1), E_extra)
    edges += [(int(x), int(y)) for x, y in zip(a, b) if x < y]
    if cycle and V >= 8:
        edges += [(V - 6, V - 5), (V - 5, V - 4), (V - 4, V - 6), (V - 4, V - 3), (V - 2, V - 2)]
    rp, col = _csr(V, edges)
    hd = (rng.random(V) < 0.5).astype(np.uint8)
    if col.size:
        hd[np.unique(col)] = 1
    return rp, col, hd


def _check(planner, O, rp, col, hd, cont=None, nodes=None):
    perm, level, order, ncyc, placed = planner.plan_stage(rp, col, hd, cont, nodes)
    assert np.array_equal(perm, O.legacy_order(hd))
    el, eo, en = O.levelize(rp, col, hd)
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en
    if nodes is None:
        assert placed is None
        return level
    first, count, assign, reason, after = placed
    ef, ec, _ = O.feasibility(cont, nodes, want_bitmap=False)
    assert np.array_equal(first, ef) and np.array_equal(count, ec)
    ea, er, eafter, _ = O.place(cont, nodes, level=el)
    assert np.array_equal(assign, ea) and np.array_equal(reason, er)
    for i in (0, 1, 3):
        assert np.array_equal(after[i], eafter[i])
    return level


@pytest.mark.parametrize("V,E_extra,N", [(1, 0, 0), (2, 0, 0), (3, 2, 0), (3, 2, 1), (40, 60, 7), (63, 150, 64),
                                         (64, 200, 64), (64, 200, 65), (65, 30, 3), (300, 2000, 64),
                                         (511, 4000, 65), (512, 7000, 4096), (513, 500, 100), (700, 100, 0)])
def test_plan_stage_vs_oracle(V, E_extra, N, planner, O, opts):
    rp, col, hd = _stage(V, E_extra, seed=V + N)
    if N:
        cont, _ = O.gen_scenario(0x5EED1000 + V, 0, V, 1, 7)
        _, nodes = O.gen_scenario(0x5EED2000 + N, 0, 1, N, 7)
        # a small stage's servers: shrink them so some services are rejected NOFIT
        nodes = (nodes[0] // 8, nodes[1] // 8) + tuple(nodes[2:])
    else:
        cont = nodes = None
    lv = _check(planner, O, rp, col, hd, cont, nodes)
    if V >= 8:
        assert (lv == NONE).sum() >= 4  # the cycle, its tail and the self loop are CYCLE
    for mode in (2, 0):  # k_plan_small without the one-wave path; the general path: the same outputs
        opts(level_small=mode)
        _check(planner, O, rp, col, hd, cont, nodes)


@pytest.mark.parametrize("E", [255, 256, 257])
def test_plan_stage_tiny_edge_limit(E, planner, O, opts):
    """The one-wave path takes at most 256 edges (u8 columns): 255 / 256 in it, 257 past it; duplicate
    edges and a self loop included; the tag-polled results of consecutive calls stay distinct."""
    V = 64
    rng = np.random.default_rng(E)
    a = rng.integers(0, V - 1, E - 1)
    b = np.minimum(a + 1 + rng.integers(0, 9, E - 1), V - 1)
    edges = list(zip(a.tolist(), b.tolist())) + [(40, 40)]
    rp, col = _csr(V, edges)
    hd = (rng.random(V) < 0.7).astype(np.uint8)
    for _ in range(300):  # > 255 calls: the 8-bit tag wraps
        _check(planner, O, rp, col, hd)
    opts(level_small=2)
    _check(planner, O, rp, col, hd)


def test_plan_stage_tiny_corrupt_inputs(planner):
    """Corrupt CSRs on the one-wave path: a column >= V (also one that a u8 cannot hold), a row_ptr
    that does not end at E, a decreasing row and a row_ptr value past 16 bits -- FP_ECORRUPT, nothing
    written, and the next call is fine."""
    from fleetflow_amd import _lib
    from fleetflow_amd._lib import FleetplaceError
    cases = [([0, 1, 2], [0, 2]), ([0, 1, 2], [0, 300]), ([0, 1, 1], [1, 0]), ([0, 2, 1], [1, 0]),
             ([0, 70000, 2], [1, 0])]
    for rp, col in cases:
        with pytest.raises(FleetplaceError) as ei:
            planner.plan_stage(np.array(rp, np.uint32), np.array(col, np.uint32), np.array([1, 1], np.uint8))
        assert ei.value.code == _lib.FP_ECORRUPT, (rp, col)
    p, lv, od, nc, _ = planner.plan_stage([0, 1, 1], [1], [0, 1])
    assert p.tolist() == [0, 1] and lv.tolist() == [0, 1] and od.tolist() == [0, 1] and nc == 0


def test_plan_stage_limits_edges(planner, O):
    """The edge limit: 8192 edges in one kernel, 8193 on the general path."""
    for E in (8192, 8193):
        V = 400
        rng = np.random.default_rng(E)
        a = rng.integers(0, V - 1, E)
        b = np.minimum(a + 1 + rng.integers(0, 20, E), V - 1)
        rp, col = _csr(V, list(zip(a.tolist(), b.tolist())))
        hd = np.ones(V, np.uint8)
        _check(planner, O, rp, col, hd)


def test_plan_stage_zero_demand_and_cordon(planner, O):
    """Zero-demand services on a table whose first servers are cordoned; label and port conflicts."""
    V, N = 20, 6
    rp, col = _csr(V, [(0, 1), (1, 2), (5, 6)])
    hd = np.zeros(V, np.uint8)
    hd[[1, 2, 6]] = 1
    cpu = np.array([0] * 8 + [100] * 12, np.uint32)
    mem = np.array([0] * 8 + [64] * 12, np.uint32)
    req = np.array([0, 1, 2, 0] * 5, np.uint32)
    conf = np.array([1, 0, 0, 1 << 16, 2] * 4, np.uint32)
    nodes = (np.array([500] * N, np.uint32), np.array([512] * N, np.uint32),
             np.array([3, 1, 2, 3, 0, 3], np.uint32), np.zeros(N, np.uint32),
             np.array([0, 0, 1, 1, 1, 1], np.uint8))
    _check(planner, O, rp, col, hd, (cpu, mem, req, conf), nodes)


def test_plan_stage_rejects_corrupt_csr_writes_nothing(planner):
    from fleetflow_amd import _lib
    from fleetflow_amd._lib import FleetplaceError
    import ctypes as ct
    rp, col, hd = np.array([0, 1, 2], np.uint32), np.array([0, 7], np.uint32), np.array([0, 1], np.uint8)
    with pytest.raises(FleetplaceError) as ei:
        planner.plan_stage(rp, col, hd)
    assert ei.value.code == _lib.FP_ECORRUPT
    # nothing written on error
    perm = np.full(2, 7, np.uint32)
    level = np.full(2, 7, np.uint32)
    order = np.full(2, 7, np.uint32)
    g = _lib.FpGraph(2, 2, rp.ctypes.data, col.ctypes.data, hd.ctypes.data)
    u32 = _lib.u32p
    rc = planner._L.fp_plan_stage(planner._ctx, ct.byref(g), None, None, perm.ctypes.data_as(u32),
                                  level.ctypes.data_as(u32), order.ctypes.data_as(u32), None, None, None, None, None)
    assert rc == _lib.FP_ECORRUPT
    assert (perm == 7).all() and (level == 7).all() and (order == 7).all()
    # the context is still usable
    p, lv, od, nc, _ = planner.plan_stage([0, 1, 1], [1], [0, 1])
    assert p.tolist() == [0, 1] and lv.tolist() == [0, 1] and od.tolist() == [0, 1] and nc == 0


def test_plan_stage_dry_run_fixtures(kats, planner):
    """The config-1 dry-run fixtures through flow.plan_stage (one fp_plan_stage call per stage)."""
    from fleetflow_amd.flow import Flow, Service, Stage, plan_stage
    for fx in kats["dry_run_fixtures"]:
        flow = Flow(services={n: Service(depends_on=d) for n, d in fx["depends_on"].items()},
                    stages={fx["stage"]: Stage(services=fx["services"], servers=fx["servers"])})
        plan = plan_stage(flow, fx["stage"], planner)
        assert plan.order == fx["order"], fx["source"]
        assert [plan.levels[n] for n in fx["services"]] == fx["levels"], fx["source"]
