"""GPU: bounded global links between pipeline segments (fp_pipe.hip `gring_wait`).

When every segment of a launch is resident at once (one scenario, or few small ones),
a segment-to-segment link is a fixed ring with back-pressure instead of storage for
every container, so the workspace no longer grows with segments x containers.  These
tests force tiny rings (a producer stalls on its consumer every few slots) and check
the plan bit-exact against the C oracle, bound the workspace of the north-star sizes,
and check 2M containers x 200k nodes against oracle digests (tests/golden/
ffd_big_digest.json, made by tests/golden/make_big_digest.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0700
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "ffd_big_digest.json")


def _check(planner, O, cont, nodes):
    assign, reason, after = planner.place(cont, nodes)
    ea, er, eafter, _ = O.place(cont, nodes)
    assert np.array_equal(assign, ea)
    assert np.array_equal(reason, er)
    for i in (0, 1, 3):
        assert np.array_equal(after[i], eafter[i])


@pytest.mark.parametrize("slots", ["8", "9", "64"])
@pytest.mark.parametrize("C,N", [(60_000, 12_000), (20_000, 30_000)])
def test_small_ring_single_scenario(C, N, slots, planner, O, opts):
    """One scenario, narrow geometry (segments of four one-group stages: 47-118
    segments), links of 8/9/64 slots of 64 containers."""
    opts(link_slots=int(slots))
    assert planner.geometry(1, C, N)["bounded"] == 1
    cont, nodes = O.gen_scenario(SEED + C + N, 0, C, N, 7)
    _check(planner, O, cont, nodes)


@pytest.mark.parametrize("w,seg", [("4", "4"), ("1", "12"), ("1", "32")])
def test_small_ring_batch(w, seg, planner, O, opts):
    """A few scenarios (all segments resident: lag 0, bounded links) in the narrow and
    one-wave geometries, 8-slot rings."""
    opts(link_slots=8, pipe_w=int(w), pipe_seg=int(seg))
    S, C, N, base = 4, 12_000, 6_000, 3
    assert planner.geometry(S, C, N)["bounded"] == 1
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED + 5, base + s, C, N, 7)
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
        for i in (0, 1, 3):
            assert np.array_equal(after[i][s * N:(s + 1) * N], eafter[i])


def test_workspace_bounded(planner):
    """Config 3 (1M x 100k, 390 links) and 2M x 200k (781 links) take well under 1 GB of
    workspace; round 1 sized every link for every container (~9.4 GB for config 3)."""
    ws3 = planner.place_ws_bytes(1, 1_000_000, 100_000)
    ws2m = planner.place_ws_bytes(1, 2_000_000, 200_000)
    assert 0 < ws3 < 0.5e9, ws3
    assert 0 < ws2m < 1.0e9, ws2m
    assert planner.place_ws_bytes(0, 10, 10) == 0


def _sha(a, dt):
    return hashlib.sha256(np.ascontiguousarray(a.astype(dt)).tobytes()).hexdigest()


def test_2m_x_200k_vs_oracle_digest(planner, O):
    """2M containers x 200k nodes, one scenario (782 segments over bounded links):
    bit-exact against the oracle's plan, node state and cost, via committed digests."""
    with open(GOLDEN) as f:
        cases = json.load(f)["cases"]
    for case in cases:
        C, N = case["C"], case["N"]
        cont, nodes = O.gen_scenario(case["seed"], case["scenario"], C, N, case["flags"])
        assign, reason, after = planner.place(cont, nodes)
        idx = np.asarray(case["sample_index"])
        assert assign[idx].astype(np.int64).tolist() == case["sample_assign"]
        assert int((reason != 0).sum()) == case["n_rejected"]
        assert int(O.cost(assign, N, case["scenario"])) == case["cost"]
        assert _sha(assign, np.uint32) == case["assign_sha256"]
        assert _sha(reason, np.uint8) == case["reason_sha256"]
        assert _sha(after[0], np.uint32) == case["cpu_free_sha256"]
        assert _sha(after[1], np.uint32) == case["mem_free_sha256"]
        assert _sha(after[3], np.uint32) == case["conflict_used_sha256"]
