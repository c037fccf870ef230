"""GPU parity of the packed-capacity FFD kernels (fp_pipe_pk.h).

When every cpu and every mem value of a batch is a multiple of 2^sc and below 2^(15 + sc), the
FFD kernels hold (cpu, mem) in one guarded 32-bit word and test both with one subtraction.  The
decision is made on the device from the batch's OR words; fp_ctx_place_path reports which kernel
ran.  Every shape below has a packed twin (fp_pipe_tus.h) and runs both ways -- packed (auto) and
u32 (FP_OPT_PACKED = 0) -- against the oracle: assignment, reason, packed cost and node state.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0077
NONE = 0xFFFFFFFF


def _batch(O, S, C, N, flags=7, base=0, seed=SEED):
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(seed, base + s, C, N, flags)
        conts.append(c)
        nodes.append(n)
    return conts, nodes


def _check_batch(planner, O, conts, nodes, base=0):
    S, C, N = len(conts), conts[0][0].size, nodes[0][0].size
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)], scen_base=base)
    path = planner.place_path()

    def one(s):
        ea, er, eafter, _ = O.place(conts[s], nodes[s])
        ok = (np.array_equal(assign[s * C:(s + 1) * C], ea) and np.array_equal(reason[s * C:(s + 1) * C], er)
              and int(cost[s]) == O.cost(ea, N, base + s)
              and all(np.array_equal(after[i][s * N:(s + 1) * N], eafter[i]) for i in (0, 1, 3)))
        return s, ok

    with ThreadPoolExecutor(16) as ex:
        bad = [s for s, ok in ex.map(one, range(S)) if not ok]
    assert not bad, f"scenarios differing from the oracle: {bad[:10]}"
    return path


# (S, C, N) -> the geometry's kernel pair (pipe_geom): n1 one-group stages, m10 4 x 10 groups,
# m8 2 x 8 groups, w12 one-wave 12 groups (five waves), big the six-wave 12-group kernel
SHAPES = {"n1": (1, 20_000, 3_000), "n1-multi": (3, 4_000, 700), "m10": (64, 3_000, 5_000),
          "m8": (600, 1_000, 5_000), "w12": (1_100, 500, 5_000), "big": (4_096, 200, 768)}
KERNEL = {"n1": (1, 4), "n1-multi": (1, 4), "m10": (10, 4), "m8": (8, 2), "w12": (12, 1), "big": (12, 1)}


@pytest.mark.parametrize("packed", [None, 0])
@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_packed_and_u32_kernels_match_the_oracle(shape, packed, planner, O, opts):
    S, C, N = SHAPES[shape]
    geo = planner.geometry(S, C, N)
    assert (geo["groups"], geo["stages"]) == KERNEL[shape], geo
    if packed is not None:
        opts(packed=packed)
    conts, nodes = _batch(O, S, C, N, base=5)
    path = _check_batch(planner, O, conts, nodes, base=5)
    assert path["ran"]
    assert path["packed"] == (packed is None), path  # generator values pack (cpu / 2, mem / 64)


def _scenario(rng, C, N, cpu_vals, mem_vals, node_cpu, node_mem):
    cpu = rng.choice(cpu_vals, C).astype(np.uint32)
    mem = rng.choice(mem_vals, C).astype(np.uint32)
    req = np.where(rng.random(C) < 0.2, 1 << rng.integers(0, 4, C), 0).astype(np.uint32)
    conf = np.where(rng.random(C) < 0.2, 1 << rng.integers(0, 32, C), 0).astype(np.uint32)
    cf = rng.choice(node_cpu, N).astype(np.uint32)
    mf = rng.choice(node_mem, N).astype(np.uint32)
    lab = rng.integers(0, 16, N).astype(np.uint32)
    sc = (rng.random(N) < 0.95).astype(np.uint8)
    return (cpu, mem, req, conf), (cf, mf, lab, np.zeros(N, np.uint32), sc)


@pytest.mark.parametrize("case", ["max-field", "shift-9", "one-past", "odd-low-bit", "exact-fits"])
@pytest.mark.parametrize("S,C,N", [(1, 6_000, 500), (4_096, 100, 768)])
def test_packed_range_boundaries(case, S, C, N, planner, O):
    """The packing decision at its edges: the largest packed field (0x7FFF after the shift), a shift
    of 9, one value past the range (u32 kernel), a single odd value (shift 0), and demands equal to
    whole free capacities (the subtraction's zero result, no borrow)."""
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    if case == "max-field":
        args = ([2, 4, 100, 30000], [2, 8, 64], [65534, 32768, 60000], [0x7FFF * 2, 4096])
        expect = True
    elif case == "shift-9":
        args = ([512 * k for k in (1, 3, 7, 60)], [1024, 2048], [512 * 0x7FFF, 512 * 100], [512 * 0x7FFF])
        expect = True
    elif case == "one-past":
        args = ([2, 4, 100], [2, 8], [65536, 4000], [4096])  # 65536 >> 1 = 0x8000
        expect = False
    elif case == "odd-low-bit":
        args = ([3, 4, 100], [2, 8], [30000, 4000], [4096])  # shift 0, all below 0x8000
        expect = True
    else:
        args = ([1000, 500, 250], [1024, 512], [1000, 2000], [1024, 2048])
        expect = True
    conts, nodes = [], []
    for _ in range(S):
        c, n = _scenario(rng, C, N, *args)
        conts.append(c)
        nodes.append(n)
    path = _check_batch(planner, O, conts, nodes)
    assert path["packed"] == expect, path


def test_packed_full_u32_fields_take_the_u32_kernel(planner, O):
    """Full-range values never pack: the u32 kernel runs, still exact."""
    big = 0xFFFFFFFF
    conts = [(np.array([big, big - 1, 0, 7], np.uint32), np.array([big, 0, big, 7], np.uint32),
              np.array([big, 0, 1, 0], np.uint32), np.array([big, 0, 0, 0], np.uint32))]
    nodes = [(np.array([big, big, 9], np.uint32), np.array([big, big, 9], np.uint32),
              np.array([big, 1, 0], np.uint32), np.zeros(3, np.uint32), np.ones(3, np.uint8))]
    path = _check_batch(planner, O, conts, nodes)
    assert path["ran"] and not path["packed"]
