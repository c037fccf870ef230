"""Synthetic workloads of SPEC.md section 3 on the host (numpy), for the benchmark's inputs.

The container / node generator runs on the device (fp_dev_gen_batch); the config-5
depends_on DAG (SPEC.md 3.3) is built here: `n_chains` chains of `chain_len`, `n_layers`
fan-out layers of `layer_width` vertices that depend on 1-4 earlier vertices, `n_cycles`
injected 3-cycles in the last layer, every id pushed through a Fisher-Yates permutation.
Output: the reversed CSR (row d lists the vertices depending on d, in logical edge order)
and has_deps, as fleetplace.h `fp_graph` takes it.  tests/test_synth.py checks it against
the C oracle's generator (oracle/fp_oracle.c fpo_gen_dag) on the same seed.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
TAG_DAG = 0xDADADADADADADADA
M64 = (1 << 64) - 1


def draw(seed: int, idx):
    """SPEC.md 3.1: the (idx+1)-th SplitMix64 output from state `seed`, vectorised over idx."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & M64) + (np.asarray(idx, np.uint64) + np.uint64(1)) * GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def dag_vertices(n_chains, chain_len, n_layers, layer_width):
    return n_chains * chain_len + n_layers * layer_width


def gen_dag(seed: int, n_chains: int, chain_len: int, n_layers: int, layer_width: int, n_cycles: int):
    s = (seed ^ TAG_DAG) & M64
    nc = n_chains * chain_len
    V = dag_vertices(n_chains, chain_len, n_layers, layer_width)
    deps, dents = [], []
    # chains: vertex i of chain k depends on vertex i - 1
    if chain_len > 1:
        k = np.arange(n_chains, dtype=np.int64)[:, None] * chain_len
        i = np.arange(1, chain_len, dtype=np.int64)[None, :]
        deps.append((k + i - 1).ravel())
        dents.append((k + i).ravel())
    # fan-out layers, in logical order: vertex v depends on m = 1 + draw(k) % 4 pool members
    for L in range(n_layers):
        pool = nc + L * layer_width
        v = nc + L * layer_width + np.arange(layer_width, dtype=np.int64)
        if pool == 0:
            continue
        kk = v.astype(np.uint64) * np.uint64(8)
        m = (np.uint64(1) + draw(s, kk) % np.uint64(4)).astype(np.int64)
        q = np.arange(4, dtype=np.int64)[None, :]
        take = q < m[:, None]                                        # [width, 4], row-major = logical order
        d = (draw(s, kk[:, None] + np.uint64(1) + q.astype(np.uint64)) % np.uint64(pool)).astype(np.int64)
        deps.append(d[take])
        dents.append(np.broadcast_to(v[:, None], take.shape)[take])
    # 3-cycles among the last layer's first vertices: a -> b -> c -> a in depends_on terms
    if n_layers > 0 and layer_width >= 3:
        base = nc + (n_layers - 1) * layer_width
        nq = min(n_cycles, layer_width // 3)  # q with 3q + 2 < layer_width
        a = base + 3 * np.arange(nq, dtype=np.int64)
        b, c = a + 1, a + 2
        deps.append(np.stack([b, c, a], 1).ravel())
        dents.append(np.stack([a, b, c], 1).ravel())
    dep = np.concatenate(deps) if deps else np.zeros(0, np.int64)
    dent = np.concatenate(dents) if dents else np.zeros(0, np.int64)
    # Fisher-Yates permutation: j = draw(s', i) % i for i = V..2
    perm = np.arange(V, dtype=np.int64)
    if V > 1:
        iv = np.arange(V, 1, -1, dtype=np.uint64)
        js = (draw((s ^ 0x1111111111111111) & M64, iv) % iv).astype(np.int64)
        pl = perm.tolist()
        for i, j in zip(range(V, 1, -1), js.tolist()):
            pl[i - 1], pl[j] = pl[j], pl[i - 1]
        perm = np.asarray(pl, np.int64)
    pd, pt = perm[dep], perm[dent]
    # reversed CSR: row d = the dependents of d, edges of a row in logical order (stable sort)
    order = np.argsort(pd, kind="stable")
    col = pt[order].astype(np.uint32)
    row_ptr = np.zeros(V + 1, np.uint32)
    np.cumsum(np.bincount(pd, minlength=V), out=row_ptr[1:])
    has_deps = np.zeros(V, np.uint8)
    has_deps[pt] = 1
    return row_ptr, col, has_deps
