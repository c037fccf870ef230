"""Ordering consumers driven by GPU levels.

The reference starts a stage's services one by one in ``order_by_dependencies``
order (crates/fleetflow-container/src/engine.rs:355-452, order from :157).  The
planner's levels turn that into parallel start waves (plan_output.start_waves):
every in-set ``depends_on`` edge must cross from an earlier wave to a later one,
CYCLE vertices must be in no wave, and every other vertex in exactly one."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NONE = 0xFFFFFFFF
SEED = 0x5EED0000


def _check_waves(waves, names_to_idx, row_ptr, col, level):
    V = level.size
    wave_of = np.full(V, -1, np.int64)
    for k, wave in enumerate(waves):
        idx = np.fromiter((names_to_idx(n) for n in wave), np.int64, len(wave))
        assert (wave_of[idx] == -1).all(), "vertex in two waves"
        wave_of[idx] = k
    cyc = level == NONE
    assert (wave_of[cyc] == -1).all(), "CYCLE vertex scheduled"
    assert (wave_of[~cyc] >= 0).all(), "vertex in no wave"
    src = np.repeat(np.arange(V), np.diff(row_ptr.astype(np.int64)))
    dst = col.astype(np.int64)
    live = ~cyc[src] & ~cyc[dst]
    assert (wave_of[src][live] < wave_of[dst][live]).all(), "a depends_on edge does not cross to a later wave"
    # a vertex downstream of a cycle is itself CYCLE (SPEC.md 2.2)
    assert not (cyc[src] & ~cyc[dst]).any()
    return wave_of


def test_config5_levels_to_start_waves(planner, O):
    """BASELINE config 5's 1M-vertex DAG: GPU levels -> start waves; every edge crosses."""
    from fleetflow_amd.flow import Plan
    from fleetflow_amd.plan_output import start_waves
    rp, col, hd = O.gen_dag(SEED + 5, 1000, 500, 50, 10_000, 333)
    level, order, ncyc = planner.levelize(rp, col, hd)
    assert ncyc == 999
    V = hd.size
    names = [f"v{i}" for i in range(V)]
    plan = Plan("live", [], dict(zip(names, level.tolist())), [names[i] for i in order.tolist()], {}, {})
    waves = start_waves(plan)
    assert len(waves) == int(level[level != NONE].max()) + 1 - (0 if (level == 0).any() else 1)
    wave_of = _check_waves(waves, lambda n: int(n[1:]), rp, col, level)
    # waves keep declaration order inside a wave
    for wave in waves[:3] + waves[-3:]:
        idx = [int(n[1:]) for n in wave]
        assert idx == sorted(idx)
    assert wave_of.max() == len(waves) - 1


def test_flow_plan_start_waves_end_to_end(planner, O):
    """A 20k-service stage built as a Flow (names, depends_on strings, deps outside the
    stage, a self-dependency): plan_stage on the GPU -> start waves -> wave script."""
    from fleetflow_amd.flow import Flow, Service, Stage, plan_stage, stage_graph
    from fleetflow_amd.plan_output import start_waves, wave_start_script
    rp, col, hd = O.gen_dag(SEED + 55, 40, 100, 8, 2000, 5)
    V = hd.size
    deps = [[] for _ in range(V)]
    for d in range(V):
        for v in col[rp[d]:rp[d + 1]]:
            deps[int(v)].append(f"s{d}")
    rng = np.random.default_rng(5)
    for v in rng.integers(0, V, 50):
        deps[int(v)].append("external-db")   # outside the target set: satisfied
    deps[7] = deps[7] + ["s7"]                 # self-dependency -> CYCLE
    services = {f"s{i}": Service(depends_on=deps[i]) for i in range(V)}
    names = list(services)
    flow = Flow(services=services, stages={"live": Stage(services=names)})
    plan = plan_stage(flow, "live", planner)
    waves = start_waves(plan)
    _, _, row_ptr, cl, has_deps = stage_graph(names, flow)
    level = np.array([plan.levels[n] for n in names], np.uint32)
    el, _, _ = O.levelize(row_ptr, cl, has_deps)
    assert np.array_equal(level, el)
    assert level[7] == NONE
    _check_waves(waves, lambda n: int(n[1:]), row_ptr, cl, level)
    script = wave_start_script(plan, "proj")
    assert len(script) == len(waves) and script[0].startswith("  wave 0: proj-live-")


def test_config5b_full_size_placement(planner, O):
    """BASELINE config 5b at full size: the GPU levels of the 1M-vertex DAG
    feed the placement of its 1M containers on 100k nodes (999 CYCLE members skipped).  Assign,
    reason and the final node state must be the oracle's, given the oracle's own levels."""
    seed5 = SEED + 5  # bench.py SEED5
    rp, col, hd = O.gen_dag(seed5, 1000, 500, 50, 10_000, 333)
    level, _, ncyc = planner.levelize(rp, col, hd)
    el, _, en = O.levelize(rp, col, hd)
    assert ncyc == en == 999 and np.array_equal(level, el)
    V, N = hd.size, 100_000
    cont, nodes = O.gen_scenario(seed5, 0, V, N, 7)
    assign, reason, after = planner.place(cont, nodes, level=level)
    ea, er, eafter, _ = O.place(cont, nodes, level=el)
    assert int((reason == 2).sum()) == 999
    assert np.array_equal(assign, ea)
    assert np.array_equal(reason, er)
    for i in (0, 1, 3):
        assert np.array_equal(after[i], eafter[i])
