"""GPU parity: every HIP path, called through the C ABI, is bit-exact with the CPU
oracle on the same seeded inputs, the reference's known answers and the golden
fixtures; full-size configs are checked through size-independent invariants."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NONE = 0xFFFFFFFF
SEED = 0x5EED0000


def _flow(case):
    from fleetflow_amd.flow import Flow, Service
    return Flow(services={n: Service(depends_on=d) for n, d in case["depends_on"].items()})


# ---- A1 legacy order ----------------------------------------------------------------
def test_order_by_dependencies_reference_kats(kats, planner):
    from fleetflow_amd.flow import order_by_dependencies
    for case in kats["order_by_dependencies"]:
        assert order_by_dependencies(case["services"], _flow(case), planner) == case["expected"], case["source"]


@pytest.mark.parametrize("small", [1, 0])
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 1023, 1024, 1025, 100_000, 1_000_000])
def test_legacy_order_random(n, small, planner, O, opts):
    """Up to 1024 vertices the partition is one launch (k_part_small); FP_OPT_LEVEL_SMALL = 0 keeps
    the three-kernel path there too."""
    opts(level_small=small)
    rng = np.random.default_rng(n)
    hd = (rng.random(n) < 0.37).astype(np.uint8)
    if n == 0:
        assert planner.legacy_order(hd).size == 0
        return
    assert np.array_equal(planner.legacy_order(hd), O.legacy_order(hd))


# ---- A2 levels -----------------------------------------------------------------------
def test_levels_known_answers(kats, planner):
    from fleetflow_amd.flow import levelize_stage
    for case in kats["levels_expected"]:
        levels, order = levelize_stage(case["services"], _flow(case), planner)
        assert levels == case["levels"], case["source"]
        assert order == case["level_order"], case["source"]


def test_levelize_golden(golden, planner):
    for case in golden["levelize"]:
        level, order, ncyc = planner.levelize(case["row_ptr"], case["col"], case["has_deps"])
        assert level.tolist() == case["level"] and order.tolist() == case["order"]
        assert ncyc == sum(1 for x in case["level"] if x == NONE)


@pytest.mark.parametrize("small", [1, 0])
@pytest.mark.parametrize("params", [(20, 30, 6, 50, 3), (0, 0, 4, 100, 5), (200, 3, 2, 300, 0), (1, 1, 0, 0, 0),
                                    (4, 50, 3, 100, 4)])
def test_levelize_random_dags(params, small, planner, O):
    """Generated DAGs, through the one-launch small-graph levelizer (<= 512 vertices) and with it
    off (FP_OPT_LEVEL_SMALL = 0: the asynchronous path)."""
    rp, col, hd = O.gen_dag(SEED + sum(params), *params)
    planner.set_option("level_small", small)
    try:
        level, order, ncyc = planner.levelize(rp, col, hd)
    finally:
        planner.set_option("level_small")
    el, eo, en = O.levelize(rp, col, hd)
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


def _csr(V, edges):
    edges = sorted(edges, key=lambda t: t[0])  # stable: per-dep order kept
    rp = np.zeros(V + 1, np.uint32)
    for d, _ in edges:
        rp[d + 1] += 1
    rp = np.cumsum(rp).astype(np.uint32)
    col = np.array([t for _, t in edges], np.uint32)
    return rp, col


@pytest.mark.parametrize("shape", ["star", "dup_and_self", "long_chain_fanout", "wide_hubs"])
def test_levelize_async_shapes(shape, planner, O):
    """Shapes aimed at the asynchronous levelizer's paths: wave-cooperative expansion
    (a vertex with thousands of dependents), duplicate edges and self loops (CAS
    retries, CYCLE), chain continuation with fan-out side edges, many hubs."""
    rng = np.random.default_rng(7)
    if shape == "star":
        V = 20_000
        edges = [(0, v) for v in range(1, V)] + [(v, v + 1) for v in range(1, 200)]
    elif shape == "dup_and_self":
        V = 3000
        edges = [(v, v + 1) for v in range(0, V - 1, 2)] * 2 + [(5, 5), (17, 17)]
        edges += [(int(a), int(b)) for a, b in zip(rng.integers(0, V // 2, 2000), rng.integers(V // 2, V, 2000))]
    elif shape == "long_chain_fanout":
        V = 30_000
        edges = [(v, v + 1) for v in range(0, 5000)]
        edges += [(int(a), int(b)) for a, b in zip(rng.integers(0, 5000, 40_000), rng.integers(5001, V, 40_000))]
    else:
        V = 50_000
        hubs = rng.integers(0, 100, 200_000)
        edges = [(int(h), int(t)) for h, t in zip(hubs, rng.integers(100, V, 200_000))]
        edges += [(int(t), int(t) + 1) for t in range(100, V - 1, 3)]
    rp, col = _csr(V, edges)
    hd = np.zeros(V, np.uint8)
    hd[np.unique(col)] = 1
    hd[rng.integers(0, V, V // 10)] = 1  # deps outside the target set
    level, order, ncyc = planner.levelize(rp, col, hd)
    el, eo, en = O.levelize(rp, col, hd)
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


@pytest.mark.parametrize("shape", ["ring_with_tails", "join_then_chain", "random_forest", "cycle_fed_tree",
                                   "chain_big_side_fans"])
def test_levelize_only_parent_shapes(shape, planner, O):
    """Only-parent structures for k_lvl_async's chain hops: rings of only-parent edges with chains
    hanging off them (never final), a deep chain below a join, a 200k-vertex random forest, a
    tree fed by a cycle member, and a chain whose vertices pass on 300-2000 side edges each as
    partial items (round 5 capped a partial's skip at 256 edges; 16-B entries carry any range),
    half of the side children leaves (final where they become ready, never queued)."""
    rng = np.random.default_rng(11)
    if shape == "ring_with_tails":
        V = 20_000
        edges = [(v, (v + 1) % 1000) for v in range(1000)]            # a 1000-ring, in-degree 1 each
        edges += [(int(a), int(b)) for a, b in zip(rng.integers(0, 1000, 300), range(1000, 1300))]
        edges += [(v, v + 1) for v in range(1300, 5000)]              # a chain from a source
        edges += [(int(a), int(b)) for a, b in zip(rng.integers(1000, 5000, 8000), rng.integers(5000, V, 8000))]
    elif shape == "join_then_chain":
        V = 12_000
        edges = [(0, 2), (1, 2)] + [(v, v + 1) for v in range(2, 6000)]
        edges += [(int(a), int(b)) for a, b in zip(rng.integers(2, 6000, 9000), rng.integers(6000, V, 9000))]
    elif shape == "random_forest":
        V = 200_000
        par = (rng.random(V - 1) * np.arange(1, V)).astype(np.int64)  # parent < child: a forest
        edges = list(zip(par.tolist(), range(1, V)))
        edges += [(int(a), int(b)) for a, b in zip(rng.integers(0, V // 2, 2000), rng.integers(V // 2, V, 2000)) if a < b]
    elif shape == "chain_big_side_fans":
        V = 60_000
        edges = [(v, v + 1) for v in range(0, 3000)]                  # first edges: the chain
        for v in range(0, 3000, 97):                                  # hop vertices with big fans
            fan = int(rng.integers(300, 2000))
            edges += [(v, int(t)) for t in rng.integers(3001, V, fan)]
        edges += [(int(a), int(b)) for a, b in zip(rng.integers(3001, 30_000, 20_000), rng.integers(30_000, V, 20_000))]
    else:
        V = 9_000
        edges = [(0, 1), (1, 2), (2, 0), (3, 0)]                      # 0 has two parents (3 and 2)
        edges += [(2, 4)] + [(v, v + 1) for v in range(4, 4000)]      # below the cycle: never final
        edges += [(5000 + i, 5001 + i) for i in range(3000)] + [(7000, 300), (8500, 8600)]
    rp, col = _csr(V, edges)
    hd = np.zeros(V, np.uint8)
    hd[np.unique(col)] = 1
    hd[rng.integers(0, V, V // 7)] = 1
    level, order, ncyc = planner.levelize(rp, col, hd)
    el, eo, en = O.levelize(rp, col, hd)
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


@pytest.mark.parametrize("sync,sort", [(0, 1), (1, 1), (0, 0)])
@pytest.mark.parametrize("chain", [1022, 1023, 1024, 1025])
def test_levelize_start_order_sort_limits(chain, sync, sort, planner, O):
    """The start order's counting sort (fp_order.hip `level_sort`) takes at most 1024 keys
    (levels + the cycle key); longer graphs take the radix sort.  Chains around that limit,
    over 19 ragged counting-sort tiles with side edges, a 3-cycle, both schedules, and the
    radix sort forced (FP_OPT_LEVEL_SORT = 0)."""
    rng = np.random.default_rng(chain)
    V = 300_001
    edges = [(v, v + 1) for v in range(chain - 1)]
    a, b = rng.integers(0, V, 60_000), rng.integers(0, V, 60_000)
    edges += [(int(x), int(y)) for x, y in zip(a, b) if chain <= x < y]  # max level = chain - 1 exactly
    edges += [(V - 3, V - 2), (V - 2, V - 1), (V - 1, V - 3)]
    rp, col = _csr(V, edges)
    hd = np.zeros(V, np.uint8)
    hd[np.unique(col)] = 1
    planner.set_option("levelize_sync", sync)
    planner.set_option("level_sort", sort)
    try:
        level, order, ncyc = planner.levelize(rp, col, hd)
    finally:
        planner.set_option("levelize_sync")
        planner.set_option("level_sort")
    el, eo, en = O.levelize(rp, col, hd)
    assert en >= 3
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


def test_levelize_async_unpacked_entries(planner, O):
    """V >= 2^24: round 5 packed queue entries as (level << 8 | skip) and ran this size without
    partial hand-off; the 16-B entries of round 6 carry the level and the edge range whole, so the
    same path runs at every size.  Same levels and order as the oracle."""
    rng = np.random.default_rng(3)
    V = (1 << 24) + 100
    heads = rng.integers(0, V - 600, 40)
    edges = [(int(h) + i, int(h) + i + 1) for h in heads for i in range(500)]
    edges += [(int(h), int(t)) for h, t in zip(rng.integers(0, V, 3000), rng.integers(0, V, 3000)) if h < t]
    edges = sorted(set(edges))
    rp, col = _csr(V, edges)
    hd = np.zeros(V, np.uint8)
    hd[np.unique(col)] = 1
    level, order, ncyc = planner.levelize(rp, col, hd)
    el, eo, en = O.levelize(rp, col, hd)
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


def test_levelize_config5_full_size(planner, O):
    """BASELINE config 5: 1M vertices (1000 chains x 500 + 50 layers x 10k), 333 3-cycles."""
    rp, col, hd = O.gen_dag(SEED + 5, 1000, 500, 50, 10_000, 333)
    level, order, ncyc = planner.levelize(rp, col, hd)
    el, eo, en = O.levelize(rp, col, hd)
    assert ncyc == en == 999
    assert np.array_equal(level, el) and np.array_equal(order, eo)


@pytest.mark.parametrize("V", [511, 512, 513])
def test_levelize_small_graph_limits(V, planner, O):
    """Around the small-graph limit (512 vertices, fp_order.hip k_lvl_small): a chain as deep as
    the graph (levels up to V with has_deps), fan-out side edges, a 3-cycle with a tail behind it,
    duplicate edges and a self loop."""
    rng = np.random.default_rng(V)
    edges = [(v, v + 1) for v in range(V - 8)]
    edges += [(int(a), int(b)) for a, b in zip(rng.integers(0, V - 8, 300), rng.integers(0, V - 8, 300)) if a < b]
    edges += [(V - 6, V - 5), (V - 5, V - 4), (V - 4, V - 6), (V - 4, V - 3), (V - 2, V - 2), (0, 3), (0, 3)]
    rp, col = _csr(V, edges)
    hd = np.zeros(V, np.uint8)
    hd[np.unique(col)] = 1
    hd[0] = 1
    level, order, ncyc = planner.levelize(rp, col, hd)
    el, eo, en = O.levelize(rp, col, hd)
    assert en == 5  # the 3-cycle, its tail, the self loop
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


def test_levelize_rejects_corrupt_csr(planner):
    from fleetflow_amd._lib import FleetplaceError
    with pytest.raises(FleetplaceError):
        planner.levelize([0, 1, 2], [0, 7], [0, 1])      # col out of range
    with pytest.raises(FleetplaceError):
        planner.levelize([0, 2, 1], [1, 0], [0, 1])      # row_ptr not monotone


# ---- A5 static server resolution / config 1 ----------------------------------------------
def test_resolve_target_server_kats(kats, planner):
    from fleetflow_amd.flow import Flow, Service, Stage, resolve_target_server
    for case in kats["resolve_target_server"]:
        flow = Flow(services={s: Service() for s in case["services"]},
                    stages={"live": Stage(services=case["services"], servers=case["servers"])})
        assert resolve_target_server(flow, "live", planner) == case["expected"], case["source"]
    assert resolve_target_server(Flow(), "missing", planner) is None


def test_dry_run_fixtures(kats, planner):
    from fleetflow_amd.flow import Flow, Service, Stage, plan_stage
    for fx in kats["dry_run_fixtures"]:
        flow = Flow(services={n: Service(depends_on=d) for n, d in fx["depends_on"].items()},
                    stages={fx["stage"]: Stage(services=fx["services"], servers=fx["servers"])})
        plan = plan_stage(flow, fx["stage"], planner)
        assert plan.order == fx["order"]
        assert [plan.levels[s] for s in fx["services"]] == fx["levels"]
        assert plan.assignment == {} and plan.rejected == {}  # no servers -> "local"


def test_dry_run_from_kdl(kats, planner):
    """Config 1 end to end: fleet.kdl -> KDL front end -> GPU plan -> dry-run text."""
    import os
    from fleetflow_amd.flow import plan_stage
    from fleetflow_amd.parser import parse_kdl_file
    from fleetflow_amd.plan_output import format_up_dry_run, plan_from_json, plan_to_json
    here = os.path.dirname(os.path.abspath(__file__))
    files = {"local": ("readme", 0), "default": ("hello-world", 1)}
    for fx in kats["dry_run_fixtures"]:
        proj, _ = files[fx["stage"]]
        flow = parse_kdl_file(os.path.join(here, "golden", "kdl", proj, ".fleetflow", "fleet.kdl"))
        assert flow.stages[fx["stage"]].services == fx["services"]
        plan = plan_stage(flow, fx["stage"], planner)
        assert plan.order == fx["order"]
        assert [plan.levels[s] for s in fx["services"]] == fx["levels"]
        assert plan.assignment == {} and plan.rejected == {}
        assert plan_from_json(plan_to_json(plan)) == plan
        text = format_up_dry_run(flow, fx["stage"], plan)
        assert text.count("    配置先: local") == len(fx["services"])


def test_plan_stage_with_registry_nodes(planner, O):
    """Registry rows -> node table -> per-service fan-out, checked against the oracle."""
    from fleetflow_amd.flow import Flow, LabelDict, Service, Stage, plan_stage
    from fleetflow_amd.registry import node_table
    rows = [{"slug": f"node-{i:02d}", "capacity": {"cpu_cores": 2 + i % 3, "memory_gb": 4 + 2 * (i % 2)},
             "labels": {"region": "tokyo" if i % 2 else "osaka"}, "scheduling": "cordon" if i == 3 else None}
            for i in range(6)]
    nodes = node_table(rows)
    svcs = {f"s{i}": Service(cpu_m=500 + 250 * (i % 5), mem_mib=1024 * (1 + i % 3),
                             labels=["region=tokyo"] if i % 4 == 0 else [],
                             anti_affinity="web" if i % 3 == 0 else None, depends_on=[f"s{i - 1}"] if i else [])
            for i in range(20)}
    flow = Flow(services=svcs, stages={"live": Stage(services=list(svcs))})
    plan = plan_stage(flow, "live", planner, servers=nodes)
    ld = LabelDict([lab for s in svcs.values() for lab in s.labels] + [lab for n in nodes for lab in n.labels])
    cont = ([s.cpu_m for s in svcs.values()], [s.mem_mib for s in svcs.values()],
            [ld.mask(s.labels) for s in svcs.values()], [(1 << 16) if s.anti_affinity else 0 for s in svcs.values()])
    nd = ([n.cpu_m for n in nodes], [n.mem_mib for n in nodes], [ld.mask(n.labels) for n in nodes],
          [0] * len(nodes), [int(n.schedulable) for n in nodes])
    ea, er, _, _ = O.place(cont, nd, level=[plan.levels[s] for s in svcs])
    for i, s in enumerate(svcs):
        if ea[i] != NONE:
            assert plan.assignment[s] == nodes[ea[i]].slug
        else:
            assert plan.rejected[s] == "NOFIT"
    # the dry-run's stage-2 candidates (first feasible server and count on the pristine table)
    ef, ec, _ = O.feasibility(cont, nd, want_bitmap=False)
    for i, s in enumerate(svcs):
        assert plan.candidates[s] == (int(ec[i]), nodes[ef[i]].slug if ef[i] != NONE else None), s
        if ec[i] == 0:  # count 0 on the pristine table: rejected NOFIT by the placement too
            assert plan.rejected[s] == "NOFIT"
    from fleetflow_amd.plan_output import format_up_dry_run, plan_from_json, plan_to_json
    assert plan_from_json(plan_to_json(plan)) == plan
    assert format_up_dry_run(flow, "live", plan).count("    配置候補: ") == len(svcs)


# ---- A6 FFD ------------------------------------------------------------------------------
def test_ffd_golden(golden, planner, O):
    for case in golden["ffd"]:
        s = O.scenario_seed(case["seed"], case["scenario"])
        cont = O.gen_containers(s, case["C"], case["flags"])
        nodes = O.gen_nodes(s, case["N"])
        assign, reason, after = planner.place(cont, nodes, level=case["level"])
        assert assign.tolist() == case["assign"], case["name"]
        assert reason.tolist() == case["reason"], case["name"]
        assert [after[0].tolist(), after[1].tolist(), after[3].tolist()] == case["nodes_after"]


def _check_ffd(planner, O, cont, nodes, level=None):
    assign, reason, after = planner.place(cont, nodes, level=level)
    ea, er, eafter, _ = O.place(cont, nodes, level=level)
    assert np.array_equal(assign, ea)
    assert np.array_equal(reason, er)
    for i in (0, 1, 3):
        assert np.array_equal(after[i], eafter[i])
    return assign, reason


@pytest.mark.parametrize("C,N,flags", [(1, 1, 7), (64, 64, 7), (65, 63, 7), (1000, 100, 7), (3000, 300, 1),
                                       (2000, 9500, 7), (1500, 12_000, 7)])
def test_ffd_random_vs_oracle(C, N, flags, planner, O):
    cont, nodes = O.gen_scenario(SEED + C + N, 0, C, N, flags)
    _check_ffd(planner, O, cont, nodes)


def test_ffd_edge_cases(planner, O):
    rng = np.random.default_rng(1)
    # zero-demand containers must not land on unschedulable nodes; req labels; conflicts
    C, N = 300, 50
    cont = (np.zeros(C, np.uint32), np.zeros(C, np.uint32), rng.integers(0, 4, C).astype(np.uint32),
            (1 << rng.integers(0, 32, C)).astype(np.uint32) * (rng.random(C) < 0.5))
    nodes = (rng.integers(0, 5, N).astype(np.uint32), rng.integers(0, 5, N).astype(np.uint32),
             rng.integers(0, 4, N).astype(np.uint32), np.zeros(N, np.uint32),
             (rng.random(N) < 0.6).astype(np.uint8))
    _check_ffd(planner, O, cont, nodes)
    # no nodes at all: everything NOFIT
    a, r, _ = planner.place(([5, 6], [1, 1], [0, 0], [0, 0]), ([], [], [], [], []))
    assert a.tolist() == [NONE, NONE] and r.tolist() == [1, 1]
    # no containers
    a, r, _ = planner.place(([], [], [], []), ([1], [1], [0], [0], [1]))
    assert a.size == 0
    # cycles are not placed
    a, r, _ = planner.place(([1, 1, 1], [1, 1, 1], [0, 0, 0], [0, 0, 0]), ([9], [9], [0], [0], [1]),
                            level=[0, NONE, 1])
    assert a.tolist() == [0, NONE, 0] and r.tolist() == [0, 2, 0]
    # max-value fields (full u32 range)
    big = 0xFFFFFFFF
    _check_ffd(planner, O, ([big, big - 1, 0], [big, 0, big], [big, 0, 1], [big, 0, 0]),
               ([big, big], [big, big], [big, 1], [0, 0], [1, 1]))


def test_ffd_batch_vs_oracle(planner, O):
    S, C, N, flags, base = 7, 700, 90, 7, 100
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED, base + s, C, N, flags)
        conts.append(c)
        nodes.append(n)
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)], scen_base=base)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea)
        assert np.array_equal(reason[s * C:(s + 1) * C], er)
        assert int(cost[s]) == O.cost(ea, N, base + s)
        assert np.array_equal(after[0][s * N:(s + 1) * N], eafter[0])


def test_config2_full_size(planner, O):
    """BASELINE config 2: 10k services x 1k servers, cpu/mem/port constraints."""
    cont, nodes = O.gen_scenario(SEED + 2, 0, 10_000, 1_000, 1)
    _check_ffd(planner, O, cont, nodes)


def test_config4_scenarios_full_size(planner, O):
    """BASELINE config 4 shape (50k x 5k per scenario), a few scenarios, via the device API."""
    import torch
    from fleetflow_amd import DevBatch
    S, C, N, base = 3, 50_000, 5_000, 4093
    db = DevBatch.allocate(S, C, N, "cuda:0", scen_base=base)
    planner.dev_gen_batch(SEED + 4, db, 7)
    torch.cuda.synchronize()
    for s in range(S):  # device generator == oracle generator
        ec, en = O.gen_scenario(SEED + 4, base + s, C, N, 7)
        got = [t[s * C:(s + 1) * C].cpu().numpy().view(np.uint32) for t in (db.cpu, db.mem, db.req, db.conf)]
        assert all(np.array_equal(g, e) for g, e in zip(got, ec))
        gn = [t[s * N:(s + 1) * N].cpu().numpy() for t in (db.cf, db.mf, db.lab, db.cu, db.sched)]
        assert all(np.array_equal(g.view(e.dtype), e) for g, e in zip(gn, en))
    planner.dev_place_batch(db)
    planner.sync()
    for s in range(S):
        ec, en = O.gen_scenario(SEED + 4, base + s, C, N, 7)
        ea, er, eafter, _ = O.place(ec, en)
        assert np.array_equal(db.assign[s * C:(s + 1) * C].cpu().numpy().view(np.uint32), ea)
        assert np.array_equal(db.reason[s * C:(s + 1) * C].cpu().numpy(), er)
        assert int(db.cost[s].item()) == O.cost(ea, N, base + s)
    best = torch.empty(1, dtype=torch.int32, device="cuda:0")
    planner.dev_argmin_cost(db.cost, best)
    costs = [int(x) for x in db.cost.cpu().numpy().view(np.uint64)]
    assert int(best.item()) == int(np.argmin(costs))


def test_place_batch_no_containers(planner):
    """C == 0 with S > 0: nothing placed, and every scenario's cost is still written
    (0 rejected, 0 nodes used, its own id; SPEC.md 2.4)."""
    S, N, base = 3, 40, 9
    nodes = [np.full(S * N, 100, np.uint32), np.full(S * N, 100, np.uint32), np.zeros(S * N, np.uint32),
             np.zeros(S * N, np.uint32), np.ones(S * N, np.uint8)]
    empty = np.zeros(0, np.uint32)
    assign, reason, cost, after = planner.place_batch(S, 0, N, [empty] * 4, nodes, scen_base=base)
    assert assign.size == 0 and reason.size == 0
    assert [int(c) for c in cost] == [base + s for s in range(S)]
    assert np.array_equal(after[0], nodes[0])


def test_place_batch_scenario_id_limit(planner):
    """scen_base + S > 65536 would wrap the packed cost's 16-bit id: refused."""
    from fleetflow_amd._lib import FP_EOVERFLOW, FleetplaceError
    one = [np.ones(2, np.uint32)] * 4
    nodes = [np.full(2, 9, np.uint32), np.full(2, 9, np.uint32), np.zeros(2, np.uint32), np.zeros(2, np.uint32),
             np.ones(2, np.uint8)]
    planner.place_batch(2, 1, 1, one, nodes, scen_base=65534)
    with pytest.raises(FleetplaceError) as e:
        planner.place_batch(2, 1, 1, one, nodes, scen_base=65535)
    assert e.value.code == FP_EOVERFLOW


def test_config4_bench_size_batch(planner, O):
    """The bench geometry at scale: 256 scenarios of 50k x 5k in one dev_place_batch
    (two segments of four 10-group stages, many tickets in flight).  Scenarios
    {0, mid, last} are checked plan-for-plan against the oracle, and the argmin
    against the oracle's costs of all 256 scenarios."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from fleetflow_amd import DevBatch
    S, C, N, base, seed = 256, 50_000, 5_000, 1024, SEED + 4
    db = DevBatch.allocate(S, C, N, "cuda:0", scen_base=base)
    planner.dev_gen_batch(seed, db, 7)
    planner.dev_place_batch(db)
    planner.sync()
    costs = db.cost.cpu().numpy().view(np.uint64)

    def oracle_cost(s):
        cont, nodes = O.gen_scenario(seed, base + s, C, N, 7)
        ea, er, _, _ = O.place(cont, nodes)
        return s, ea, er, O.cost(ea, N, base + s)

    with ThreadPoolExecutor(16) as ex:
        res = list(ex.map(oracle_cost, range(S)))
    for s, ea, er, ec in res:
        assert int(costs[s]) == ec, s
        if s in (0, S // 2, S - 1):
            assert np.array_equal(db.assign[s * C:(s + 1) * C].cpu().numpy().view(np.uint32), ea), s
            assert np.array_equal(db.reason[s * C:(s + 1) * C].cpu().numpy(), er), s
    best = torch.empty(1, dtype=torch.int32, device="cuda:0")
    planner.dev_argmin_cost(db.cost, best)
    assert int(best.item()) == int(np.argmin([r[3] for r in res]))
    del db
    torch.cuda.empty_cache()


@pytest.mark.parametrize("case", ["all_equal", "cpu_const", "mem_const", "rank_limit", "past_rank_limit",
                                  "dense_wide", "zero_mix"])
def test_ffd_sort_key_compression(case, planner, O):
    """The LDS sort ranks a scenario's values into digits when it has at most 256 distinct
    values per dimension, all below 2^18 (fp_place.hip k_scen_sort), and sorts the raw values
    otherwise (its generic fallback); either way the order, and so the plan, must be the oracle's."""
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    C, N = 3000, 400
    lim = 1 << 18
    cpu = rng.integers(1, 5000, C)
    mem = rng.integers(1, 20000, C)
    if case == "all_equal":
        cpu[:] = 700; mem[:] = 900
    elif case == "cpu_const":
        cpu[:] = 1234
    elif case == "mem_const":
        mem[:] = 77
    elif case == "rank_limit":
        cpu[:5] = lim - 1; mem[-5:] = lim - 1
    elif case == "past_rank_limit":
        cpu[:5] = lim; mem[-5:] = lim - 1
    elif case == "dense_wide":
        cpu = rng.integers(0, lim, C); mem = rng.integers(0, lim, C)
    elif case == "zero_mix":
        cpu[::3] = 0; mem[::5] = 0
    cont = (cpu.astype(np.uint32), mem.astype(np.uint32), np.zeros(C, np.uint32),
            (rng.random(C) < 0.2).astype(np.uint32) << rng.integers(0, 32, C).astype(np.uint32))
    big = int(max(cpu.max(), mem.max())) * 4 + 10
    nodes = (rng.integers(0, big, N).astype(np.uint32), rng.integers(0, big, N).astype(np.uint32),
             np.zeros(N, np.uint32), np.zeros(N, np.uint32), (rng.random(N) < 0.95).astype(np.uint8))
    _check_ffd(planner, O, cont, nodes)
    # and batched (scenario field in the key), scenarios with different value sets
    S = 5
    conts = [tuple(np.roll(a, 17 * s) if i < 2 else a for i, a in enumerate(cont)) for s in range(S)]
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [np.tile(a, S) for a in nodes], scen_base=0)
    for s in range(S):
        ea, er, _, _ = O.place(conts[s], nodes)
        assert np.array_equal(assign[s * C:(s + 1) * C], ea)
        assert np.array_equal(reason[s * C:(s + 1) * C], er)


def test_ffd_sort_rank_keys_u64(planner, O):
    """~140k distinct cpu and mem values below 2^18: the rank fields need 18 + 18 bits, so
    the rank keys go to the u64 sort (fp_place.hip); the plan must still be the oracle's."""
    rng = np.random.default_rng(11)
    C, N = 140_000, 300
    cpu = rng.permutation(1 << 18)[:C].astype(np.uint32)
    mem = rng.permutation(1 << 18)[:C].astype(np.uint32)
    cont = (cpu, mem, np.zeros(C, np.uint32), np.zeros(C, np.uint32))
    nodes = (rng.integers(1 << 18, 1 << 22, N).astype(np.uint32), rng.integers(1 << 18, 1 << 22, N).astype(np.uint32),
             np.zeros(N, np.uint32), np.zeros(N, np.uint32), np.ones(N, np.uint8))
    _check_ffd(planner, O, cont, nodes)


# ---- segmented pipeline: N beyond one workgroup's LDS (> 80 groups of 64 nodes) ----
@pytest.mark.parametrize("C,N,flags", [(20_000, 6_000, 7), (30_000, 20_000, 7), (2_000, 100_000, 7),
                                       (60_000, 33_000, 3), (5_000, 5_121, 7)])
def test_ffd_segments_vs_oracle(C, N, flags, planner, O):
    """Segments of one scenario hand their unplaced containers downstream through
    global rings; the plan must be the sequential first fit all the same."""
    cont, nodes = O.gen_scenario(SEED + 3 * C + N, 1, C, N, flags)
    _check_ffd(planner, O, cont, nodes)


def test_ffd_segments_batch_and_cycles(planner, O):
    S, C, N, base = 3, 4_000, 11_000, 17
    conts, nodes, levels = [], [], []
    rng = np.random.default_rng(5)
    for s in range(S):
        c, n = O.gen_scenario(SEED + 9, base + s, C, N, 7)
        conts.append(c)
        nodes.append(n)
        levels.append(np.where(rng.random(C) < 0.01, NONE, 0).astype(np.uint32))
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)],
                                                      level=np.concatenate(levels), scen_base=base)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s], level=levels[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea)
        assert np.array_equal(reason[s * C:(s + 1) * C], er)
        assert int(cost[s]) == O.cost(ea, N, base + s)
        for i in (0, 1, 3):
            assert np.array_equal(after[i][s * N:(s + 1) * N], eafter[i])


def test_config3_full_size(planner, O):
    """BASELINE config 3: 1M containers x 100k nodes with label anti-affinity, one
    scenario (the narrow geometry: 391 segments of four one-group stages), bit-exact
    against the oracle at full size."""
    cont, nodes = O.gen_scenario(SEED + 3, 0, 1_000_000, 100_000, 7)
    assign, reason = _check_ffd(planner, O, cont, nodes)
    assert (reason == 1).any() and (reason == 0).any()


# ---- stage 2 feasibility --------------------------------------------------------------------
def test_feasibility_golden(golden, planner, O):
    for case in golden["feasibility"]:
        s = O.scenario_seed(case["seed"], 0)
        cont = O.gen_containers(s, case["C"], case["flags"])
        nodes = O.gen_nodes(s, case["N"])
        first, count, bm = planner.feasibility(cont, nodes)
        assert first.tolist() == case["first"] and count.tolist() == case["count"]
        assert [f"{int(w):016x}" for w in bm] == case["bitmap_hex"]


@pytest.mark.parametrize("C,N", [(1, 1), (200, 5000), (5000, 200), (64, 70_000), (3333, 3333)])
def test_feasibility_random_vs_oracle(C, N, planner, O):
    cont, nodes = O.gen_scenario(SEED + 7 * C + N, 1, C, N, 7)
    rng = np.random.default_rng(C)
    cf = nodes[0] - rng.integers(0, 3000, N).clip(0, nodes[0]).astype(np.uint32)
    cu = (rng.random(N) < 0.3).astype(np.uint32) << rng.integers(0, 32, N).astype(np.uint32)
    nodes = (cf, nodes[1], nodes[2], cu, nodes[4])
    first, count, bm = planner.feasibility(cont, nodes)
    ef, ec, eb = O.feasibility(cont, nodes)
    assert np.array_equal(first, ef) and np.array_equal(count, ec) and np.array_equal(bm, eb)


# ---- pipeline geometry: "one-wave" (one-wave segments of up to 32 groups) is what many
# scenarios get, "narrow" (segments of 4, stages of 1 group) what a few small ones get;
# "wide" (4 stages of 10 groups) was round 1's many-scenario geometry, "one-wave-40" the
# 64-bit group-set path (> 32 groups); all are forced here so every size runs through each
GEOMETRIES = {"wide": ("4", "40"), "narrow": ("4", "4"), "one-stage": ("1", "16"), "one-wave": ("1", "32"),
              "one-wave-40": ("1", "40")}


@pytest.fixture(params=sorted(GEOMETRIES))
def geometry(request, opts):
    w, seg = GEOMETRIES[request.param]
    opts(pipe_w=int(w), pipe_seg=int(seg))
    return request.param


@pytest.mark.parametrize("C,N,flags", [(4000, 640, 7), (4000, 641, 7), (7000, 2560, 7), (7000, 2561, 7),
                                       (5000, 5120, 7), (3000, 5121, 3), (64, 64, 7), (1000, 100, 7)])
def test_ffd_geometry_edges(C, N, flags, planner, O, geometry):
    """Stage (64 / 640 nodes), segment (256 / 2560) and two-segment (5120) boundaries."""
    cont, nodes = O.gen_scenario(SEED + 13 * C + N, 3, C, N, flags)
    _check_ffd(planner, O, cont, nodes)


def test_ffd_batch_geometries(planner, O, geometry):
    S, C, N, base = 5, 3000, 1500, 7
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED + 21, base + s, C, N, 7)
        conts.append(c)
        nodes.append(n)
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)], scen_base=base)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea)
        assert np.array_equal(reason[s * C:(s + 1) * C], er)
        assert int(cost[s]) == O.cost(ea, N, base + s)


@pytest.mark.parametrize("N", [700, 3000])
def test_ffd_zero_demand_mixed(N, planner, O, geometry):
    """All-zero containers among ordinary ones; the first tiles (and scattered nodes) are
    unschedulable, so zero containers must skip whole stages; some containers use only labels
    or only conflicts with zero cpu/mem."""
    rng = np.random.default_rng(N)
    C = 5000
    cont, nodes = O.gen_scenario(SEED + 77, 1, C, N, 7)
    cpu, mem, req, conf = (np.array(a, np.uint32) for a in cont)
    z = rng.random(C) < 0.05          # all-zero
    cpu[z] = mem[z] = req[z] = conf[z] = 0
    lab_only = (~z) & (rng.random(C) < 0.03)
    cpu[lab_only] = mem[lab_only] = 0
    conf[lab_only] = 0
    conf_only = (~z) & (~lab_only) & (rng.random(C) < 0.03)
    cpu[conf_only] = mem[conf_only] = 0
    req[conf_only] = 0
    conf[conf_only] = (1 << rng.integers(0, 32, int(conf_only.sum()))).astype(np.uint32)
    cf, mf, lab, cu, sc = (np.array(a) for a in nodes)
    sc = sc.astype(np.uint8)
    sc[:650] = 0                      # whole first stage (and part of the second) cordoned
    sc[rng.random(N) < 0.1] = 0
    _check_ffd(planner, O, (cpu, mem, req, conf), (cf, mf, lab, cu, sc))
    # nothing schedulable at all: zero containers are NOFIT too
    _check_ffd(planner, O, (cpu[:300], mem[:300], req[:300], conf[:300]), (cf, mf, lab, cu, np.zeros(N, np.uint8)))


@pytest.mark.parametrize("n_lab", [32, 64, 100])
@pytest.mark.parametrize("N", [5, 64])
def test_label_only_containers_count_their_node(n_lab, N, planner, O):
    """a one-group stage's systolic fill counts the nodes whose records changed,
    and a label-only container (cpu = mem = conf = 0, req != 0) changes none.  Here >= 32 of them
    (a systolic queue) fit only node 3, which nothing else uses: the packed cost must count node 3
    (n_nodes_used, SPEC.md 2.4) exactly as the oracle does.  Also the serial loop (threshold 64)."""
    S, base, k = 3, 11, 20
    conts, nodes = [], []
    for s in range(S):
        cpu = [5 + s] * k + [0] * n_lab
        mem = [7] * k + [0] * n_lab
        req = [0] * k + [1 << 4] * n_lab
        conf = [0] * (k + n_lab)
        conts.append(tuple(np.array(x, np.uint32) for x in (cpu, mem, req, conf)))
        lab = np.zeros(N, np.uint32)
        lab[3] = 1 << 4
        nodes.append((np.full(N, 1000, np.uint32), np.full(N, 1000, np.uint32), lab, np.zeros(N, np.uint32),
                       np.ones(N, np.uint8)))
    C = k + n_lab
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    for sys_thr in (None, 64):
        planner.set_option("systolic", sys_thr if sys_thr is not None else -1)  # -1: FP_OPT_AUTO
        try:
            assign, reason, cost, _ = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                          [cat(nodes, i) for i in range(5)], scen_base=base)
        finally:
            planner.set_option("systolic")
        for s in range(S):
            ea, er, _, _ = O.place(conts[s], nodes[s])
            assert np.array_equal(assign[s * C:(s + 1) * C], ea)
            assert np.array_equal(reason[s * C:(s + 1) * C], er)
            assert int(cost[s]) == O.cost(ea, N, base + s), (s, sys_thr)
            assert 3 in set(ea.tolist())


def test_forced_bounded_geometry_reports_the_launched_kernel(planner, opts):
    """a 4096-scenario batch runs the six-wave kernel only with unbounded links; a
    forced bounded ring runs the five-wave one, and fp_place_geometry's resident slots must be that
    kernel's (the same 12-group one-wave kernel a 2048-scenario batch runs)."""
    auto = planner.geometry(4096, 50_000, 5_000)
    five = planner.geometry(2048, 50_000, 5_000)
    assert auto["groups"] == five["groups"] == 12 and auto["stages"] == five["stages"] == 1
    assert not auto["bounded"]
    opts(link_bounded=1)
    forced = planner.geometry(4096, 50_000, 5_000)
    assert forced["bounded"] == 1
    assert forced["resident"] == five["resident"] < auto["resident"]


@pytest.mark.parametrize("S,C,N", [(3, 700, 300), (5, 3000, 5000), (4, 50_000, 5_000)])
def test_feasibility_batch_vs_oracle(S, C, N, planner, O):
    """Stage 2 batched over scenarios (fp_dev_feasibility_batch): every scenario's first
    feasible node and feasible-node count equal the oracle's sweep on that scenario; the
    node state is not mutated.  Half-used node states exercise the conflict/capacity tests."""
    import torch
    from fleetflow_amd import DevBatch
    base = 11
    db = DevBatch.allocate(S, C, N, "cuda:0", scen_base=base)
    planner.dev_gen_batch(SEED + 6, db, 7)
    rng = np.random.default_rng(S * C)
    cu = torch.from_numpy(((rng.random(S * N) < 0.3).astype(np.uint32) << rng.integers(0, 32, S * N).astype(np.uint32))
                          .view(np.int32)).to("cuda:0")
    db.cu.copy_(cu)
    db.cf.sub_(torch.from_numpy(rng.integers(0, 3000, S * N).astype(np.int32)).to("cuda:0")).clamp_(min=0)
    snap = [t.clone() for t in (db.cf, db.mf, db.cu)]
    first = torch.empty(S * C, dtype=torch.int32, device="cuda:0")
    count = torch.empty(S * C, dtype=torch.int32, device="cuda:0")
    planner.dev_feasibility_batch(db, first, count)
    planner.sync()
    assert all(torch.equal(a, b) for a, b in zip(snap, (db.cf, db.mf, db.cu)))
    fh, ch = first.cpu().numpy().view(np.uint32), count.cpu().numpy().view(np.uint32)
    nodes_all = [t.cpu().numpy() for t in (db.cf, db.mf, db.lab, db.cu, db.sched)]
    for s in sorted({0, S // 2, S - 1}):
        cont, _ = O.gen_scenario(SEED + 6, base + s, C, N, 7)
        nodes = tuple(a[s * N:(s + 1) * N].view(np.uint32) if a.dtype != np.uint8 else a[s * N:(s + 1) * N]
                      for a in nodes_all)
        k = min(C, 4000)  # the oracle sweep is O(C*N): a prefix of the containers at full size
        ef, ec, _ = O.feasibility(tuple(np.asarray(x)[:k] for x in cont), nodes, want_bitmap=False)
        assert np.array_equal(fh[s * C:s * C + k], ef), s
        assert np.array_equal(ch[s * C:s * C + k], ec), s


def test_levelize_deep_chain_three_sort_passes(planner, O):
    """A chain of 1,050,000 vertices: levels need 21 bits, so the start order takes three LSD
    passes of the counting sort (the key range is read on the device only); side edges and a
    3-cycle as above."""
    rng = np.random.default_rng(21)
    V, chain = 1_100_000, 1_050_000
    edges = [(v, v + 1) for v in range(chain - 1)]
    a, b = rng.integers(0, V, 20_000), rng.integers(0, V, 20_000)
    edges += [(int(x), int(y)) for x, y in zip(a, b) if chain <= x < y]
    edges += [(V - 3, V - 2), (V - 2, V - 1), (V - 1, V - 3)]
    rp, col = _csr(V, edges)
    hd = np.zeros(V, np.uint8)
    hd[np.unique(col)] = 1
    level, order, ncyc = planner.levelize(rp, col, hd)
    el, eo, en = O.levelize(rp, col, hd)
    assert int(el[el != 0xFFFFFFFF].max()) == chain - 1
    assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


@pytest.mark.parametrize("S,C,dv", [(3, 50_000, 300), (2, 20_000, 257), (4, 8_000, 256)])
def test_scen_sort_generic_fallback(S, C, dv, planner, O):
    """Scenarios that fit the per-scenario LDS sort but have more than 256 distinct cpu values
    (dv > 256) take k_scen_sort's generic LSD fallback, chosen in the workgroup (no read-back);
    dv = 256 stays on the digit path.  Plans, reasons and costs must be the oracle's either way."""
    rng = np.random.default_rng(C + dv)
    N = 2_000
    conts, nodes = [], []
    vals = rng.choice(np.arange(100, 100 + 20 * dv, 20), dv, replace=False).astype(np.uint32)
    for s in range(S):
        c, n = O.gen_scenario(SEED + 61, s, C, N, 7)
        c = [np.array(a, np.uint32) for a in c]
        c[0] = vals[rng.integers(0, dv, C)]
        c[0][:dv] = vals                               # every value present in every scenario
        conts.append(c)
        nodes.append(n)
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)], scen_base=7)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea), s
        assert np.array_equal(reason[s * C:(s + 1) * C], er), s
        assert int(cost[s]) == O.cost(ea, N, 7 + s)
        for i in (0, 1, 3):
            assert np.array_equal(after[i][s * N:(s + 1) * N], eafter[i])


def test_scen_sort_mixed_eligibility(planner, O):
    """Each workgroup of the LDS sort ranks its own scenario: in one batch, scenarios with dense
    digits (<= 256 values per dimension), with too many distinct values, with a value >= 2^18 and
    with a single value take the digit sort or the generic fallback side by side."""
    rng = np.random.default_rng(23)
    S, C, N = 8, 6000, 700
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED + 77, s, C, N, 7)
        c = [np.array(a, np.uint32) for a in c]
        kind = s % 4
        if kind == 0:    # dense digits
            c[0] = rng.choice(np.arange(50, 5000, 25), C).astype(np.uint32)
            c[1] = rng.choice(np.arange(64, 64 * 200, 64), C).astype(np.uint32)
        elif kind == 1:  # too many distinct mem values
            c[1] = rng.integers(1, 100_000, C).astype(np.uint32)
        elif kind == 2:  # one demand past the rank tables
            c[0][rng.integers(0, C)] = (1 << 18) + 5
        else:            # one value per dimension
            c[0][:] = 300; c[1][:] = 4096
        conts.append(c)
        nodes.append(n)
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)], scen_base=40)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea), s
        assert np.array_equal(reason[s * C:(s + 1) * C], er), s
        assert int(cost[s]) == O.cost(ea, N, 40 + s)
        assert np.array_equal(after[0][s * N:(s + 1) * N], eafter[0])


@pytest.mark.parametrize("V", [1021, 1022, 1025])
def test_levelize_sync_cycle_key_pass_boundary(V, planner, O):
    """The level-synchronous schedule's cycle key is iters + 2 <= V + 3: at V = 1021 /
    1022 a chain as deep as the graph makes it 1024 / 1025 -- 11 bits, two counting-sort passes, so
    the queued pass count must cover V + 3.  The general path (> 512 vertices), both schedules."""
    edges = [(v, v + 1) for v in range(V - 1)]
    rp, col = _csr(V, edges)
    hd = np.ones(V, np.uint8)
    el, eo, en = O.levelize(rp, col, hd)
    for sync in (1, 0):
        planner.set_option("levelize_sync", sync)
        try:
            level, order, ncyc = planner.levelize(rp, col, hd)
        finally:
            planner.set_option("levelize_sync")
        assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


def test_levelize_queue_reuse_across_calls(planner, O):
    """The asynchronous levelizer keeps its work queues between calls and refills them only when
    the last call left them dirty (fp_order.hip kQClean): alternate graphs, a corrupt CSR (queues
    dirty), an edgeless graph (no async kernel), bigger graphs (the buffer grows) and bigger graphs
    that still fit the buffer, every result against the oracle."""
    from fleetflow_amd._lib import FleetplaceError

    def dag(V, E, seed):
        rng = np.random.default_rng(seed)
        a, b = rng.integers(0, V, E), rng.integers(0, V, E)
        edges = [(int(x), int(y)) for x, y in zip(a, b) if x < y] + [(V - 3, V - 2), (V - 2, V - 1), (V - 1, V - 3)]
        rp, col = _csr(V, edges)
        hd = (rng.random(V) < 0.7).astype(np.uint8)
        return rp, col, hd

    # 40k -> 45k: a larger queue inside the same buffer (its capacity has 25 % slack), whose tail
    # the 40k call never used -- "clean" must cover the whole buffer (the plan_stage 513 -> 700
    # services case that once read unfilled slots and hung)
    graphs = [dag(5_000, 20_000, 1), dag(40_000, 90_000, 2), dag(45_000, 100_000, 4), "corrupt",
              dag(5_000, 20_000, 1), (np.zeros(2_001, np.uint32), np.zeros(0, np.uint32), np.ones(2_000, np.uint8)),
              dag(120_000, 300_000, 3), dag(40_000, 90_000, 2), dag(140_000, 320_000, 5)]
    for g in graphs:
        if isinstance(g, str):  # "corrupt": col out of range
            with pytest.raises(FleetplaceError):
                planner.levelize([0, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2] + [2] * 600, [1, 5000], np.ones(610, np.uint8))
            continue
        rp, col, hd = g
        level, order, ncyc = planner.levelize(rp, col, hd)
        el, eo, en = O.levelize(rp, col, hd)
        assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en


@pytest.mark.parametrize("shape", ["one_slice", "ragged_slices", "hub_child", "shift_13", "sequence"])
def test_levelize_binned_indegree(shape, planner, O):
    """The asynchronous levelizer's in-degrees binned by child range in LDS (fp_order.hip
    k_indeg_bin / k_indeg_hist) against the global-atomic count (FP_OPT_INDEG_BIN = 0) and the
    oracle: fewer edges than one 4096-edge slice, a ragged last slice, one child with 60k parents
    (one bucket, every slice), a graph whose buckets need 8192-vertex ranges (V > 4M), and the two
    paths alternating on one context (the binned count stores every in-degree, the other zeroes)."""
    from fleetflow_amd._lib import FleetplaceError
    rng = np.random.default_rng(len(shape))

    def rand(V, E):
        a, b = rng.integers(0, V, E), rng.integers(0, V, E)
        edges = [(int(x), int(y)) for x, y in zip(a, b) if x < y] + [(V - 3, V - 2), (V - 2, V - 1), (V - 1, V - 3)]
        rp, col = _csr(V, edges)
        hd = np.zeros(V, np.uint8)
        hd[np.unique(col)] = 1
        return rp, col, hd

    if shape == "one_slice":
        graphs = [rand(3_000, 2_500)]
    elif shape == "ragged_slices":
        graphs = [rand(70_000, 4096 * 9 + 77)]
    elif shape == "hub_child":
        V = 80_000
        edges = [(v, V - 1) for v in range(60_000)] + [(v, v + 1) for v in range(60_000, V - 2)]
        rp, col = _csr(V, edges)
        hd = np.zeros(V, np.uint8)
        hd[np.unique(col)] = 1
        graphs = [(rp, col, hd)]
    elif shape == "shift_13":
        graphs = [rand(4096 * 1024 + 5, 200_000)]
    else:
        graphs = [rand(50_000, 120_000), rand(20_000, 30_000), rand(50_000, 120_000)]
    for i, (rp, col, hd) in enumerate(graphs):
        el, eo, en = O.levelize(rp, col, hd)
        for on in ([1, 0] if shape != "sequence" else [i % 2, 1 - i % 2]):
            planner.set_option("indeg_bin", on)
            planner.set_option("level_small", 0)
            try:
                level, order, ncyc = planner.levelize(rp, col, hd)
            finally:
                planner.set_option("indeg_bin")
                planner.set_option("level_small")
            assert np.array_equal(level, el) and np.array_equal(order, eo) and ncyc == en, (shape, i, on)
    # a corrupt CSR on the binned path: a child out of range in the last slice, rows not monotone
    V = 5_000
    rp = np.arange(V + 1, dtype=np.uint32)
    rp[V] = V
    col = (np.arange(V, dtype=np.uint32) + 1) % V
    bad_col = col.copy()
    bad_col[-1] = V + 9
    bad_rp = rp.copy()
    bad_rp[2000] = 5
    for r, c in ((rp, bad_col), (bad_rp, col)):
        planner.set_option("level_small", 0)
        try:
            with pytest.raises(FleetplaceError):
                planner.levelize(r, c, np.ones(V, np.uint8))
        finally:
            planner.set_option("level_small")
