"""GPU parity of the per-scenario LDS sort (fp_place.hip k_scen_sort, fp_pipe.hip k_payload_lds /
k_gather_payload): scenarios of at most ~50.3k containers sort in one workgroup's LDS (digits
from the scenario's own <= 256 distinct values per dimension, else the in-workgroup generic
fallback) instead of the radix-key path.  Both paths must give the oracle's plan bit for bit; the
cases push the kernel's limits (the LDS capacity, a single bucket holding every
container, 256-value digits, equal keys in every wave, cycles)."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED5050
# largest C whose scenario fits the 160 KB of LDS: u16 index (its region also holds the rank
# tables, 96 KB) + u8 digit per container (each 16-B aligned) + 12,816 B of tables
# (fp_place.hip ss_lds_bytes)
SS_MAX_C = 50_336


@pytest.fixture(params=["scen_sort", "scen_sort_gather", "radix"])
def sort_path(request, opts):
    """The LDS sort with the LDS-chunked payload (k_payload_lds, default), with the random-gather
    payload (k_gather_payload), and the radix-key path."""
    pl = {"scen_sort_gather": 0}.get(request.param, -1)
    opts(scen_sort=0 if request.param == "radix" else -1, payload_lds=pl)
    return request.param


def _batch_check(planner, O, conts, nodes, level=None, base=0):
    S = len(conts)
    C = conts[0][0].size
    N = nodes[0][0].size
    cat = lambda parts, i: np.concatenate([p[i] for p in parts])  # noqa: E731
    lv = None if level is None else np.concatenate(level).astype(np.uint32)
    assign, reason, cost, after = planner.place_batch(S, C, N, [cat(conts, i) for i in range(4)],
                                                      [cat(nodes, i) for i in range(5)], level=lv, scen_base=base)
    for s in range(S):
        ea, er, eafter, _ = O.place(conts[s], nodes[s], level=None if level is None else level[s])
        assert np.array_equal(assign[s * C:(s + 1) * C], ea), s
        assert np.array_equal(reason[s * C:(s + 1) * C], er), s
        assert int(cost[s]) == O.cost(ea, N, base + s), s
        for i in (0, 1, 3):
            assert np.array_equal(after[i][s * N:(s + 1) * N], eafter[i]), s


def _nodes(rng, N, big=40_000):
    return (rng.integers(0, big, N).astype(np.uint32), rng.integers(0, big, N).astype(np.uint32),
            rng.integers(0, 8, N).astype(np.uint32), np.zeros(N, np.uint32),
            (rng.random(N) < 0.97).astype(np.uint8))


def _cont(rng, C, cpu_vals, mem_vals):
    return (rng.choice(cpu_vals, C).astype(np.uint32), rng.choice(mem_vals, C).astype(np.uint32),
            (rng.random(C) < 0.2).astype(np.uint32) * (1 << rng.integers(0, 3, C)).astype(np.uint32),
            (rng.random(C) < 0.2).astype(np.uint32) << rng.integers(0, 32, C).astype(np.uint32))


@pytest.mark.parametrize("case", ["generator", "one_bucket", "digits_256", "few_keys", "zero_mix", "tiny"])
def test_scen_sort_cases(case, sort_path, planner, O):
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    S, C, N = 4, 6_000, 700
    if case == "generator":
        conts, nodes = zip(*[O.gen_scenario(SEED, s, C, N, 7) for s in range(S)])
    else:
        if case == "one_bucket":      # every container the same cpu: one hd bucket of C (one wave's)
            cv, mv = np.array([1500]), np.arange(1, 257) * 37
        elif case == "digits_256":    # exactly 256 distinct values in both dimensions
            cv, mv = np.arange(1, 257) * 11, np.arange(1, 257) * 53
        elif case == "few_keys":      # long runs of equal keys inside every wave
            cv, mv = np.array([100, 2000]), np.array([64, 4096, 512])
        elif case == "zero_mix":
            cv, mv = np.array([0, 50, 100, 4000]), np.array([0, 64, 128])
        else:                         # C far below one chunk
            C = 37
            cv, mv = np.arange(1, 40) * 25, np.arange(1, 9) * 64
        conts = [_cont(rng, C, cv, mv) for _ in range(S)]
        nodes = [_nodes(rng, N) for _ in range(S)]
    _batch_check(planner, O, list(conts), list(nodes), base=3)


def test_scen_sort_bucket_register_limit(sort_path, planner, O):
    """cpu buckets of 1024 containers (the largest one a wave reorders in registers) and 1025
    (scattered straight to HBM), beside small ones."""
    rng = np.random.default_rng(77)
    S, C, N = 2, 6_000, 600
    conts = []
    for _ in range(S):
        cpu = np.concatenate([np.full(1024, 3000), np.full(1025, 2500), rng.choice(np.arange(1, 60) * 40, C - 2049)])
        cont = _cont(rng, C, [1], np.arange(1, 200) * 64)
        conts.append((rng.permutation(cpu).astype(np.uint32),) + cont[1:])
    _batch_check(planner, O, conts, [_nodes(rng, N) for _ in range(S)])


@pytest.mark.parametrize("C", [SS_MAX_C, SS_MAX_C + 1])
def test_scen_sort_lds_limit(C, planner, O):
    """At the largest C that fits LDS (per-scenario sort) and one past it (radix path)."""
    conts, nodes = zip(*[O.gen_scenario(SEED + 1, s, C, 4_000, 7) for s in range(2)])
    _batch_check(planner, O, list(conts), list(nodes))


def test_scen_sort_cycles(sort_path, planner, O):
    """CYCLE containers (level FP_NONE) ride through the payload gather's CYCLE bit."""
    rng = np.random.default_rng(5)
    S, C, N = 3, 5_000, 400
    conts, nodes = zip(*[O.gen_scenario(SEED + 2, s, C, N, 7) for s in range(S)])
    level = [np.where(rng.random(C) < 0.05, 0xFFFFFFFF, rng.integers(0, 9, C)).astype(np.uint32) for _ in range(S)]
    _batch_check(planner, O, list(conts), list(nodes), level=level)


@pytest.mark.parametrize("C", [25_600, 25_601, 40_000])
def test_scen_sort_cycles_chunks(C, sort_path, planner, O):
    """Positions across both register halves of k_payload_lds (25,600 per half) and level /
    (req, conf) arrays spanning several LDS chunks (36,864 / 18,432 containers)."""
    rng = np.random.default_rng(C)
    S, N = 2, 3_000
    conts, nodes = zip(*[O.gen_scenario(SEED + 3, s, C, N, 7) for s in range(S)])
    level = [np.where(rng.random(C) < 0.03, 0xFFFFFFFF, rng.integers(0, 5, C)).astype(np.uint32) for _ in range(S)]
    _batch_check(planner, O, list(conts), list(nodes), level=level)


def test_scen_sort_single_scenario_config2(sort_path, planner, O):
    """BASELINE config 2 (one scenario, 10k x 1k) takes the per-scenario sort too."""
    cont, nodes = O.gen_scenario(0x5EED0002, 0, 10_000, 1_000, 1)
    _batch_check(planner, O, [cont], [nodes])


@pytest.mark.parametrize("sample", ["dense", "too_many"])
def test_scen_sort_sample_value_set(sample, planner, O):
    """k_scen_sort ranks against the sample's value set (the first 8 scenarios) when it has at
    most 256 values per dimension, and a workgroup that meets a value outside it (above, below or
    between the sample's values, or >= 2^18) ranks its own scenario again (or falls back to the
    generic sort).  A sample with too many values sends every scenario to its own values."""
    rng = np.random.default_rng(0xA11 + len(sample))
    S, C, N = 16, 6_000, 700
    conts, nodes = [], []
    for s in range(S):
        c, n = O.gen_scenario(SEED + 91, s, C, N, 7)
        c = [np.array(a, np.uint32) for a in c]
        if sample == "too_many" and s == 0:
            c[0] = rng.integers(1, 100_000, C).astype(np.uint32)
        kind = s % 8 if s >= 8 else -1
        j = int(rng.integers(0, C))
        if kind == 1:
            c[0][j] = 50 * 81 + 7          # above every sample cpu value
        elif kind == 2:
            c[1][j] = 1                    # below every sample mem value
        elif kind == 3:
            c[0][j] = 50 * 40 + 25         # between two sample cpu values
        elif kind == 4:
            c[1][C - 1] = 64 * 100 + 32    # the last container of the last wave's slice
        elif kind == 5:
            c[0][j] = (1 << 18) + 3        # past the rank tables: the generic sort
        elif kind == 6:
            c[1] = rng.integers(1, 100_000, C).astype(np.uint32)  # too many values: generic
        conts.append(c)
        nodes.append(n)
    _batch_check(planner, O, conts, nodes, base=11)
