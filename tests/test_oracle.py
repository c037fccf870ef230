"""CPU tests of the oracle itself: it must reproduce the reference's own known
answers (engine.rs / provider.rs / deploy.rs tests) and the golden vectors, and
the C oracle must agree with its independent pure-Python twin."""
import numpy as np
import pytest

NONE = 0xFFFFFFFF


def _has_deps(case):
    dep = case["depends_on"]
    return [1 if (n in dep and dep[n]) else 0 for n in case["services"]]


# ---- reference-pinned known answers -------------------------------------------
def test_legacy_order_reference_kats(kats, O, P):
    for case in kats["order_by_dependencies"]:
        svcs = case["services"]
        perm_c = O.legacy_order(_has_deps(case))
        perm_py = P.legacy_order(_has_deps(case))
        assert [svcs[i] for i in perm_c] == case["expected"], case["source"]
        assert [svcs[i] for i in perm_py] == case["expected"], case["source"]
        # name-level restatement of engine.rs:67-85
        assert P.order_by_dependencies_names(svcs, case["depends_on"]) == case["expected"]


def test_levels_known_answers(kats, O, P):
    from fleetflow_amd.flow import Flow, Service, stage_graph
    for case in kats["levels_expected"]:
        flow = Flow(services={n: Service(depends_on=d) for n, d in case["depends_on"].items()})
        names, pos2v, rp, col, hd = stage_graph(case["services"], flow)
        level, order, _ = O.levelize(rp, col, hd)
        levels = [int(level[v]) for v in pos2v]
        assert levels == case["levels"], case["source"]
        lo = sorted(range(len(levels)), key=lambda i: (levels[i] == NONE, levels[i], i))
        assert [case["services"][i] for i in lo] == case["level_order"]
        lp, _ = P.levelize(len(names), list(rp), list(col), list(hd))
        assert [lp[v] for v in pos2v] == case["levels"]


def test_depth1_theorem_on_reference_tests(kats, O):
    """SPEC.md 2.2: on graphs of depth <= 1 the level order equals engine.rs's order."""
    from fleetflow_amd.flow import Flow, Service, stage_graph
    for case in kats["order_by_dependencies"][:4]:
        flow = Flow(services={n: Service(depends_on=d) for n, d in case["depends_on"].items()})
        names, pos2v, rp, col, hd = stage_graph(case["services"], flow)
        level, _, _ = O.levelize(rp, col, hd)
        lv = [int(level[v]) for v in pos2v]
        lo = sorted(range(len(lv)), key=lambda i: (lv[i], i))
        assert [case["services"][i] for i in lo] == case["expected"], case["source"]


def test_parse_plan_reference_kats(kats, P):
    for case in kats["parse_plan"]:
        assert P.parse_plan(case["plan"]) == tuple(case["expected"]), case["source"]


def test_resolve_target_server_kats(kats, O, P):
    for case in kats["resolve_target_server"]:
        assert P.resolve_target_server(case["servers"]) == case["expected"], case["source"]
        if case["servers"]:
            # the same answer from the FFD oracle with N servers, unconstrained capacity
            n, m = len(case["services"]), len(case["servers"])
            big = 0xFFFFFFFF
            assign, reason, _, _ = O.place(([0] * n, [0] * n, [0] * n, [0] * n),
                                           ([big] * m, [big] * m, [0] * m, [0] * m, [1] * m))
            assert all(case["servers"][a] == case["expected"] for a in assign)


# ---- golden vectors ---------------------------------------------------------------
def test_generator_golden(golden, O, P):
    g = golden["generator"]
    assert [P.draw(g["seed"], k) for k in range(3)] == g["draw_0_1_2"]
    s = O.scenario_seed(g["seed"], g["scenario"])
    assert s == P.scenario_seed(g["seed"], g["scenario"])
    for got, exp in zip(O.gen_containers(s, 16, 7), g["containers"]):
        assert list(got) == exp
    for got, exp in zip(O.gen_nodes(s, 16), g["nodes"]):
        assert list(got) == exp


def test_ffd_golden(golden, O):
    for case in golden["ffd"]:
        s = O.scenario_seed(case["seed"], case["scenario"])
        cont = O.gen_containers(s, case["C"], case["flags"])
        for got, exp in zip(cont, case["cont"]):
            assert list(got) == exp
        nodes = O.gen_nodes(s, case["N"])
        assign, reason, after, _ = O.place(cont, nodes, level=case["level"])
        assert list(assign) == case["assign"], case["name"]
        assert list(reason) == case["reason"], case["name"]
        assert O.cost(assign, case["N"], case["scenario"]) == case["cost"]
        for got, exp in zip((after[0], after[1], after[3]), case["nodes_after"]):
            assert list(got) == exp


def test_levelize_golden(golden, O):
    for case in golden["levelize"]:
        rp, col, hd = O.gen_dag(case["seed"], *case["params"])
        assert list(rp) == case["row_ptr"] and list(col) == case["col"] and list(hd) == case["has_deps"]
        level, order, ncyc = O.levelize(rp, col, hd)
        assert list(level) == case["level"] and list(order) == case["order"]
        assert ncyc == sum(1 for x in case["level"] if x == NONE)


def test_feasibility_golden(golden, O):
    for case in golden["feasibility"]:
        s = O.scenario_seed(case["seed"], 0)
        cont = O.gen_containers(s, case["C"], case["flags"])
        nodes = O.gen_nodes(s, case["N"])
        first, count, bm = O.feasibility(cont, nodes)
        assert list(first) == case["first"] and list(count) == case["count"]
        assert [f"{int(w):016x}" for w in bm] == case["bitmap_hex"]


# ---- C oracle == Python twin on random small instances ---------------------------------
@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_matches_python_twin(seed, O, P):
    rng = np.random.default_rng(seed)
    C, N = int(rng.integers(0, 120)), int(rng.integers(1, 40))
    flags = int(rng.integers(0, 8))
    s = P.scenario_seed(0xABC + seed, seed)
    cont = P.gen_containers(s, C, flags)
    nodes = P.gen_nodes(s, N)
    # random prior usage so conflicts/partial capacity are exercised
    cf, mf, lab, cu, sched = (list(x) for x in nodes)
    for n in range(N):
        cf[n] -= int(rng.integers(0, cf[n] // 2 + 1))
        cu[n] = int(rng.integers(0, 2 ** 32)) & int(rng.integers(0, 2 ** 32)) & int(rng.integers(0, 2 ** 32))
    level = [NONE if rng.random() < 0.05 else int(rng.integers(0, 4)) for _ in range(C)]
    a_c, r_c, after_c, _ = O.place(cont, (cf, mf, lab, cu, sched), level=level)
    cfp, mfp, cup = list(cf), list(mf), list(cu)
    a_p, r_p = P.place(*cont, cfp, mfp, lab, cup, sched, level=level)
    assert list(a_c) == a_p and list(r_c) == r_p
    assert list(after_c[0]) == cfp and list(after_c[1]) == mfp and list(after_c[3]) == cup
    f_c, n_c, b_c = O.feasibility(cont, (cf, mf, lab, cu, sched))
    f_p, n_p, b_p = P.feasibility(*cont, cf, mf, lab, cu, sched)
    assert list(f_c) == f_p and list(n_c) == n_p and [int(x) for x in b_c] == b_p


@pytest.mark.parametrize("params", [(3, 4, 2, 5, 1), (10, 3, 5, 7, 0), (1, 1, 0, 0, 0), (0, 0, 3, 6, 2)])
def test_dag_and_levels_match_twin(params, O, P):
    rp, col, hd = O.gen_dag(77, *params)
    V, rp_p, col_p, hd_p = P.gen_dag(77, *params)
    assert list(rp) == rp_p and list(col) == col_p and list(hd) == hd_p
    level, order, _ = O.levelize(rp, col, hd)
    lp, op = P.levelize(V, rp_p, col_p, hd_p)
    assert list(level) == lp and list(order) == op


def test_ffd_order_key(O, P):
    cpu = [100, 200, 200, 100, 200]
    mem = [5, 1, 9, 5, 9]
    assert list(O.ffd_order(cpu, mem)) == [2, 4, 1, 0, 3] == P.ffd_order(cpu, mem)


def test_cost_packing(O, P):
    a = [0, 0, 3, NONE, 3, 7]
    assert O.cost(a, 8, 5) == P.cost(a, 5) == (1 << 40) | (3 << 16) | 5


def test_oracle_is_thread_safe(O):
    """The bench CPU baseline and the bench-size GPU test run the oracle on many host
    threads at once: concurrent plans must equal sequential ones (the FFD sort's
    comparator state is thread-local)."""
    from concurrent.futures import ThreadPoolExecutor

    def plan(s):
        cont, nodes = O.gen_scenario(0x5EED0004, s, 4000, 400, 7)
        a, r, _, _ = O.place(cont, nodes)
        return a.tobytes() + r.tobytes()

    seq = [plan(s) for s in range(24)]
    with ThreadPoolExecutor(8) as ex:
        for _ in range(3):
            assert list(ex.map(plan, range(24))) == seq
