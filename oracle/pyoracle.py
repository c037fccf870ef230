"""Pure-Python twin of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg may
import this module, and only as the checker.  The product (fleetflow_amd /
libfleetplace.so) never imports it.

Each function restates the same reference file:line as ``oracle/fp_oracle.c``;
the twin exists so the C oracle is itself checked by an independent
implementation, and to generate small golden vectors (tests/golden/).

Parity status: ``legacy_order`` is pinned by the reference's own unit tests
(crates/fleetflow-container/src/engine.rs:603-666).  ``levelize`` and
``place`` implement semantics the reference does not have (SPEC.md 2.2/2.3):
parity against the reference is *unpinned* beyond the depth<=1 theorem and the
N=1 ``servers.first()`` special case (handlers/deploy.rs:390-398).
"""
from __future__ import annotations

NONE = 0xFFFFFFFF
OK, NOFIT, CYCLE = 0, 1, 2
M64 = (1 << 64) - 1
GAMMA = 0x9E3779B97F4A7C15
TAG_CONT = 0xC0C0C0C0C0C0C0C0
TAG_NODE = 0x5E5E5E5E5E5E5E5E
TAG_DAG = 0xDADADADADADADADA


# --- A1: crates/fleetflow-container/src/engine.rs:67-85 -----------------------
def legacy_order(has_deps):
    """Stable two-bucket partition: empty-deps-or-unknown first (:71-80), rest after (:83)."""
    first = [i for i, h in enumerate(has_deps) if not h]
    rest = [i for i, h in enumerate(has_deps) if h]
    return first + rest


def order_by_dependencies_names(services, deps_of):
    """Name-level restatement of engine.rs:67-85.

    ``deps_of`` maps a known service name to its depends_on list; names absent
    from it are unknown (they go to the first bucket, :79-80)."""
    ordered, remaining = [], []
    for name in services:
        if name in deps_of:
            (ordered if not deps_of[name] else remaining).append(name)
        else:
            ordered.append(name)
    return ordered + remaining


# --- A5: crates/fleetflow-controlplane/src/handlers/deploy.rs:390-398 ---------
def resolve_target_server(stage_servers):
    """`servers.first().cloned()` -> Option<String>; the record uses "local" for None."""
    return stage_servers[0] if stage_servers else None


# --- crates/fleetflow-cloud-sakura/src/provider.rs:15-30 -----------------------
def parse_plan(plan):
    def rust_i32(s):
        # str::parse::<i32>(): optional sign, ASCII digits, no whitespace
        if not s:
            return None
        body = s[1:] if s[0] in "+-" else s
        if not body or not all("0" <= ch <= "9" for ch in body):
            return None
        v = int(s)
        return v if -(2 ** 31) <= v < 2 ** 31 else None

    def trim_end(s, suffix):
        while suffix and s.endswith(suffix):
            s = s[: -len(suffix)]
        return s

    if plan is not None:
        parts = plan.split("-")
        if len(parts) == 2:
            core = rust_i32(trim_end(parts[0], "core"))
            mem = rust_i32(trim_end(parts[1], "gb"))
            return (1 if core is None else core, 1 if mem is None else mem)
    return (1, 1)


# --- A2: SPEC.md 2.2 -----------------------------------------------------------
def levelize(V, row_ptr, col, has_deps):
    indeg = [0] * V
    for e in range(row_ptr[V]):
        indeg[col[e]] += 1
    level = [1 if has_deps[v] else 0 for v in range(V)]
    queue = [v for v in range(V) if indeg[v] == 0]
    head = 0
    while head < len(queue):
        d = queue[head]
        head += 1
        for e in range(row_ptr[d], row_ptr[d + 1]):
            v = col[e]
            level[v] = max(level[v], level[d] + 1)
            indeg[v] -= 1
            if indeg[v] == 0:
                queue.append(v)
    for v in range(V):
        if indeg[v]:
            level[v] = NONE
    order = sorted(range(V), key=lambda v: (level[v] == NONE, level[v], v))
    return level, order


# --- A6: SPEC.md 2.3 -----------------------------------------------------------
def ffd_order(cpu, mem):
    return sorted(range(len(cpu)), key=lambda i: (-cpu[i], -mem[i], i))


def fits(c_cpu, c_mem, c_req, c_conf, cf, mf, lab, cu, sched):
    return bool(sched) and cf >= c_cpu and mf >= c_mem and (lab & c_req) == c_req and (cu & c_conf) == 0


def place(cpu, mem, req, conf, cf, mf, lab, cu, sched, level=None):
    """Returns (assign, reason); cf/mf/cu lists are mutated in place."""
    C, N = len(cpu), len(cf)
    assign = [NONE] * C
    reason = [OK] * C
    for c in ffd_order(cpu, mem):
        if level is not None and level[c] == NONE:
            reason[c] = CYCLE
            continue
        for n in range(N):
            if fits(cpu[c], mem[c], req[c], conf[c], cf[n], mf[n], lab[n], cu[n], sched[n]):
                cf[n] -= cpu[c]
                mf[n] -= mem[c]
                cu[n] |= conf[c]
                assign[c] = n
                break
        else:
            reason[c] = NOFIT
    return assign, reason


def feasibility(cpu, mem, req, conf, cf, mf, lab, cu, sched):
    C, N = len(cpu), len(cf)
    WC = (C + 63) // 64
    first, count = [NONE] * C, [0] * C
    bitmap = [0] * (WC * N)
    for c in range(C):
        for n in range(N):
            if fits(cpu[c], mem[c], req[c], conf[c], cf[n], mf[n], lab[n], cu[n], sched[n]):
                if first[c] == NONE:
                    first[c] = n
                count[c] += 1
                bitmap[(c // 64) * N + n] |= 1 << (c % 64)
    return first, count, bitmap


def cost(assign, scenario_id):
    rej = sum(1 for a in assign if a == NONE)
    used = len({a for a in assign if a != NONE})
    return (min(rej, 0xFFFFFF) << 40) | (min(used, 0xFFFFFF) << 16) | (scenario_id & 0xFFFF)


# --- SPEC.md 3: generators -------------------------------------------------------
def draw(seed, idx):
    z = (seed + (idx + 1) * GAMMA) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def scenario_seed(seed, s):
    return (seed ^ ((s * GAMMA) & M64)) & M64


def gen_containers(seed, C, flags):
    s = seed ^ TAG_CONT
    cpu, mem, req, conf = [], [], [], []
    for j in range(C):
        k = j * 8
        cpu.append(50 * (2 + draw(s, k) % 79))
        mem.append(64 * (1 + draw(s, k + 1) % 256))
        cf = rq = 0
        if (flags & 1) and draw(s, k + 2) % 1000 < 100:
            cf |= 1 << (draw(s, k + 3) % 16)
        if (flags & 2) and draw(s, k + 4) % 1000 < 200:
            cf |= 1 << (16 + draw(s, k + 5) % 16)
        if (flags & 4) and draw(s, k + 6) % 1000 < 300:
            rq = 1 << (draw(s, k + 7) % 13)
        req.append(rq)
        conf.append(cf)
    return cpu, mem, req, conf


NODE_TYPES = [(4000, 8192), (8000, 16384), (16000, 32768), (32000, 65536), (64000, 262144)]


def gen_nodes(seed, N):
    s = seed ^ TAG_NODE
    cf, mf, lab, cu, sched = [], [], [], [], []
    for n in range(N):
        k = n * 8
        t = draw(s, k) % 5
        cf.append(NODE_TYPES[t][0])
        mf.append(NODE_TYPES[t][1])
        l = (1 << (draw(s, k + 1) % 3)) | (1 << (3 + draw(s, k + 2) % 4))
        l |= (1 << (7 + draw(s, k + 3) % 4)) | (1 << (11 + draw(s, k + 4) % 2))
        lab.append(l)
        cu.append(0)
        sched.append(1 if draw(s, k + 5) % 1000 >= 20 else 0)
    return cf, mf, lab, cu, sched


def gen_dag(seed, n_chains, chain_len, n_layers, layer_width, n_cycles):
    """SPEC.md 3.3; returns (V, row_ptr, col, has_deps) as a reversed CSR."""
    s = seed ^ TAG_DAG
    n_chain_v = n_chains * chain_len
    V = n_chain_v + n_layers * layer_width
    edges = []
    for k in range(n_chains):
        for i in range(1, chain_len):
            edges.append((k * chain_len + i - 1, k * chain_len + i))
    for L in range(n_layers):
        pool = n_chain_v + L * layer_width
        for j in range(layer_width):
            v = n_chain_v + L * layer_width + j
            k = v * 8
            m = 1 + draw(s, k) % 4 if pool else 0
            for q in range(m):
                edges.append((draw(s, k + 1 + q) % pool, v))
    if n_layers > 0 and layer_width >= 3:
        base = n_chain_v + (n_layers - 1) * layer_width
        q = 0
        while q < n_cycles and 3 * q + 2 < layer_width:
            a = base + 3 * q
            edges += [(a + 1, a), (a + 2, a + 1), (a, a + 2)]
            q += 1
    sp = seed ^ TAG_DAG ^ 0x1111111111111111
    perm = list(range(V))
    for i in range(V, 1, -1):
        j = draw(sp, i) % i
        perm[i - 1], perm[j] = perm[j], perm[i - 1]
    row_ptr = [0] * (V + 1)
    has_deps = [0] * V
    for d, v in edges:
        row_ptr[perm[d] + 1] += 1
        has_deps[perm[v]] = 1
    for v in range(V):
        row_ptr[v + 1] += row_ptr[v]
    fill = row_ptr[:V]
    col = [0] * len(edges)
    for d, v in edges:
        col[fill[perm[d]]] = perm[v]
        fill[perm[d]] += 1
    return V, row_ptr, col, has_deps
