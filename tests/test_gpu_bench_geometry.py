"""GPU parity of the geometry the benchmark actually runs.

bench.py plans BASELINE config 4 as ONE fp_dev_place_batch of 4096 scenarios x 50k containers
x 5k nodes.  That batch holds more pipeline segments than the device keeps resident
(4096 x 7 > 5120), so the planner runs it with a segment ticket lag of S (segment b of every
scenario starts after phase b - 1 drained, fp_pipe.hip k_ffd_pipe) and unbounded global links.
The first test makes the exact bench call and checks every scenario's packed cost, four full
plans and the argmin against the C oracle; the others force lagged geometries on small
batches (S not a multiple of anything, 2..7 segments, the last phase) through ctx options."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED4 = 0x5EED0004  # bench.py SEED4


def _oracle_plans(O, seed, base, S, C, N, flags, threads=16):
    from concurrent.futures import ThreadPoolExecutor

    def one(s):
        cont, nodes = O.gen_scenario(seed, base + s, C, N, flags)
        ea, er, _, _ = O.place(cont, nodes)
        return ea, er, O.cost(ea, N, base + s)

    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(one, range(S)))


def test_config4_exact_bench_call(planner, O):
    """bench.py's call at N = 1: DevBatch(4096, 50k, 5k, scen_base 0), dev_gen_batch(0x5EED0004,
    flags 7), dev_place_batch.  Every cost equals the oracle's, scenarios {0, 2047, 4095, argmin}
    plan-for-plan, and the device argmin is the oracle's."""
    import torch
    from fleetflow_amd import DevBatch
    S, C, N = 4096, 50_000, 5_000
    geo = planner.geometry(S, C, N)
    assert geo["lag"] == S and geo["bounded"] == 0, geo          # phased segments, full links
    assert geo["segments"] * S > geo["resident"], geo             # more segments than slots
    db = DevBatch.allocate(S, C, N, "cuda:0", scen_base=0)
    planner.dev_gen_batch(SEED4, db, 7)
    planner.dev_place_batch(db)
    planner.sync()
    costs = db.cost.cpu().numpy().view(np.uint64)
    best = torch.empty(1, dtype=torch.int32, device="cuda:0")
    planner.dev_argmin_cost(db.cost, best)
    planner.sync()
    res = _oracle_plans(O, SEED4, 0, S, C, N, 7)
    ecost = np.array([r[2] for r in res], np.uint64)
    bad = np.nonzero(costs != ecost)[0]
    assert bad.size == 0, f"{bad.size} scenario costs differ, first {bad[:8].tolist()}"
    arg = int(np.argmin(ecost))
    assert int(best.item()) == arg
    for s in sorted({0, 2047, S - 1, arg}):
        ea, er, _ = res[s]
        assert np.array_equal(db.assign[s * C:(s + 1) * C].cpu().numpy().view(np.uint32), ea), s
        assert np.array_equal(db.reason[s * C:(s + 1) * C].cpu().numpy(), er), s
    del db
    torch.cuda.empty_cache()


# (S, groups per segment) -> 5000 nodes = 79 groups: seg 40 -> B = 2, 28 -> 3, 20 -> 4, 16 -> 5,
# 12 -> 7 (one-wave segments)
@pytest.mark.parametrize("S,seg,publish", [(5, 40, 1), (9, 28, 3), (13, 20, 8), (5, 16, 1024), (9, 12, 1),
                                            (13, 12, 8), (13, 12, 2)])
@pytest.mark.parametrize("lag", ["S", 3])
def test_forced_lag_geometries(S, seg, publish, lag, planner, O, opts):
    """Segment ticket lag forced on a small batch: ticket t -> round t / B, segment t % B,
    scenario round - segment * lag.  lag = S is the bench's phased schedule; lag 3 interleaves
    phases.  Unbounded links (a consumer may start after its producer ended), with the head
    published every `publish` full slots (1 .. the whole stream)."""
    C, N, base = 3_000, 5_000, 40
    lagv = S if lag == "S" else lag
    opts(pipe_w=1, pipe_seg=seg, pipe_lag=lagv, link_publish=publish)
    geo = planner.geometry(S, C, N)
    assert geo["lag"] == lagv and geo["bounded"] == 0 and geo["stages"] == 1, geo
    B = geo["segments"]
    assert B == -(-79 // seg), geo
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED4 + 17, base + s, C, N, 7)
        conts.append(c)
        nodes.append(n)
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)], scen_base=base)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea), (s, B)
        assert np.array_equal(reason[s * C:(s + 1) * C], er), (s, B)
        assert int(cost[s]) == O.cost(ea, N, base + s)
        for i in (0, 1, 3):
            assert np.array_equal(after[i][s * N:(s + 1) * N], eafter[i])


def test_geometry_query_defaults(planner):
    """fp_place_geometry reports what the planner picks: configs 2/3 (one scenario, narrow
    segments of four one-group stages, lag 0), config 4's shape at 256 scenarios (fits at once:
    lag 0; two segments of four 10-group stages up to 512 scenarios), at 1024 (five segments of
    two 8-group stages) and at 2048 (one-wave 12-group segments)."""
    g3 = planner.geometry(1, 1_000_000, 100_000)
    assert (g3["groups"], g3["stages"], g3["lag"]) == (1, 4, 0) and g3["segments"] == 391, g3
    g2 = planner.geometry(1, 10_000, 1_000)
    assert g2["segments"] * g2["stages"] * g2["groups"] >= 16 and g2["lag"] == 0, g2
    g4 = planner.geometry(256, 50_000, 5_000)
    assert g4["lag"] == 0 and (g4["groups"], g4["stages"], g4["segments"]) == (10, 4, 2), g4
    g4m = planner.geometry(1024, 50_000, 5_000)
    assert (g4m["groups"], g4m["stages"], g4m["segments"]) == (8, 2, 5), g4m
    g4b = planner.geometry(2048, 50_000, 5_000)
    assert (g4b["groups"], g4b["stages"], g4b["segments"]) == (12, 1, 7), g4b


# ---- systolic group fill (fp_pipe_sys.h) ------------------------------------------------------
@pytest.mark.parametrize("valu", [0, 1, 2])
@pytest.mark.parametrize("thr", [1, 24])
@pytest.mark.parametrize("C,N,flags,w,seg", [(20_000, 6_000, 7, 4, 4), (60_000, 12_000, 7, 4, 4),
                                             (4_000, 641, 7, 1, 12), (5_000, 5_121, 3, 1, 32),
                                             (30_000, 2_000, 7, 4, 40), (64, 64, 7, 4, 4),
                                             (40_000, 3_000, 7, 2, 2), (9_000, 700, 5, 1, 1)])
def test_systolic_fill_vs_oracle(C, N, flags, w, seg, thr, valu, planner, O, opts):
    """Group queues of >= thr containers take the systolic loop (thr 1: every queue), the rest
    the serial one; the plan, reasons and final node state must be the oracle's.  The systolic
    loop is compiled for stages of at most 4 groups (FP_SYS_MAX_G): wider stages report 0 and
    run the serial loop on the same inputs."""
    opts(systolic=thr, pipe_w=w, pipe_seg=seg, systolic_valu=valu)
    g = planner.geometry(1, C, N)
    assert g["systolic"] == (thr if g["groups"] <= 4 else 0), g
    cont, nodes = O.gen_scenario(SEED4 + 23 * C + N, 2, C, N, flags)
    assign, reason, after = planner.place(cont, nodes)
    ea, er, eafter, _ = O.place(cont, nodes)
    assert np.array_equal(assign, ea)
    assert np.array_equal(reason, er)
    for i in (0, 1, 3):
        assert np.array_equal(after[i], eafter[i])


@pytest.mark.parametrize("valu", [0, 1, 2])
@pytest.mark.parametrize("thr", [1, 16])
def test_systolic_batch_zero_and_cycles(thr, valu, planner, O, opts):
    """Systolic fill in a many-scenario batch with all-zero containers, cycles and cordoned
    nodes (the zero containers bypass the group loops; CYCLE members never enter)."""
    opts(systolic=thr, systolic_valu=valu)
    S, C, N, base = 6, 5_000, 3_000, 77
    rng = np.random.default_rng(thr)
    conts, nodes, levels = [], [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED4 + 31, base + s, C, N, 7)
        c = [np.array(a, np.uint32) for a in c]
        z = rng.random(C) < 0.03
        for a in c:
            a[z] = 0
        n = [np.array(a) for a in n]
        n[4] = n[4].astype(np.uint8)
        n[4][rng.random(N) < 0.1] = 0
        conts.append(c)
        nodes.append(n)
        levels.append(np.where(rng.random(C) < 0.01, 0xFFFFFFFF, 0).astype(np.uint32))
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)],
                                                      level=np.concatenate(levels), scen_base=base)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s], level=levels[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea), s
        assert np.array_equal(reason[s * C:(s + 1) * C], er), s
        assert int(cost[s]) == O.cost(ea, N, base + s)
        for i in (0, 1, 3):
            assert np.array_equal(after[i][s * N:(s + 1) * N], eafter[i])


# ---- stage-2 early-NOFIT screen (fp_pipe.hip k_node_summary) ------------------------------------
@pytest.mark.parametrize("S,C,N", [(1, 20_000, 3_000), (6, 4_000, 2_000), (64, 2_000, 640)])
def test_screen_vs_unscreened_and_oracle(S, C, N, planner, O, opts):
    """Containers whose labels lie outside every schedulable node's labels, or whose conflict bits
    every schedulable node has used, are rejected NOFIT before the pipeline.  The plans with and
    without the screen, and the oracle's, must be identical; the inputs make both rules fire (one
    scenario with every node's port 3 taken, one with no node labelled 5, cordoned nodes)."""
    base = 11
    rng = np.random.default_rng(S * C)
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED4 + 41, base + s, C, N, 7)
        c = [np.array(a, np.uint32) for a in c]
        n = [np.array(a) for a in n]
        n[4] = n[4].astype(np.uint8)
        n[4][rng.random(N) < 0.05] = 0
        if s % 3 == 0:
            n[3][:] |= 1 << 3                       # port 3 used on every node
            c[3][rng.random(C) < 0.05] |= 1 << 3
        if s % 3 == 1:
            n[2][:] &= ~np.uint32(1 << 5)           # nobody carries label bit 5
            c[2][rng.random(C) < 0.05] |= 1 << 5
        conts.append(c)
        nodes.append(n)
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    args = ([cat(conts, i) for i in range(4)], [cat(nodes, i) for i in range(5)])
    a1, r1, c1, n1 = planner.place_batch(S, C, N, *args, scen_base=base)
    opts(screen=0)
    a0, r0, c0, n0 = planner.place_batch(S, C, N, *args, scen_base=base)
    assert np.array_equal(a1, a0) and np.array_equal(r1, r0) and np.array_equal(c1, c0)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s])
        assert np.array_equal(a1[s * C:(s + 1) * C], ea), s
        assert np.array_equal(r1[s * C:(s + 1) * C], er), s
        assert int(c1[s]) == O.cost(ea, N, base + s)
        for i in (0, 1, 3):
            assert np.array_equal(n1[i][s * N:(s + 1) * N], eafter[i])
