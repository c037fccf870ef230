/*
 * fp_oracle.c -- CPU ORACLE (test infrastructure only; see fp_oracle.h header).
 *
 * Every function cites the reference file:line it restates, or SPEC.md for the
 * new semantics the north star adds (levels, FFD, generators).  Straight-line,
 * single-threaded code: clarity over speed, because this is the checker.
 */
#include "fp_oracle.h"
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* A1  crates/fleetflow-container/src/engine.rs:67-85                         */
/*   for name in services: known && !depends_on.is_empty() -> remaining,      */
/*   else (empty deps OR unknown name, :71-80) -> ordered;                    */
/*   ordered.extend(remaining) (:83).                                          */
/* ------------------------------------------------------------------------- */
void fpo_legacy_order(uint32_t n, const uint8_t *has_deps, uint32_t *perm_out) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (!has_deps[i]) perm_out[k++] = i;
    for (uint32_t i = 0; i < n; ++i)
        if (has_deps[i]) perm_out[k++] = i;
}

/* ------------------------------------------------------------------------- */
/* A2  SPEC.md 2.2: Kahn levels generalising engine.rs:67-85.                 */
/* ------------------------------------------------------------------------- */
uint32_t fpo_levelize(uint32_t V, const uint32_t *row_ptr, const uint32_t *col,
                      const uint8_t *has_deps, uint32_t *level_out, uint32_t *order_out) {
    uint32_t *indeg = (uint32_t *)calloc(V ? V : 1, sizeof(uint32_t));
    uint32_t *queue = (uint32_t *)malloc((V ? V : 1) * sizeof(uint32_t));
    for (uint32_t d = 0; d < V; ++d)
        for (uint32_t e = row_ptr[d]; e < row_ptr[d + 1]; ++e) indeg[col[e]]++;
    uint32_t head = 0, tail = 0;
    for (uint32_t v = 0; v < V; ++v) {
        level_out[v] = has_deps[v] ? 1u : 0u; /* deps outside the set: level >= 1 */
        if (indeg[v] == 0) queue[tail++] = v;
    }
    while (head < tail) {
        uint32_t d = queue[head++];
        for (uint32_t e = row_ptr[d]; e < row_ptr[d + 1]; ++e) {
            uint32_t v = col[e];
            if (level_out[d] + 1 > level_out[v]) level_out[v] = level_out[d] + 1;
            if (--indeg[v] == 0) queue[tail++] = v;
        }
    }
    uint32_t n_cycle = 0;
    for (uint32_t v = 0; v < V; ++v)
        if (indeg[v] != 0) { level_out[v] = FPO_NONE; n_cycle++; }
    /* stable counting sort by level; FPO_NONE last */
    uint32_t max_level = 0;
    for (uint32_t v = 0; v < V; ++v)
        if (level_out[v] != FPO_NONE && level_out[v] > max_level) max_level = level_out[v];
    uint32_t *cnt = (uint32_t *)calloc((size_t)max_level + 3, sizeof(uint32_t));
    for (uint32_t v = 0; v < V; ++v) {
        uint32_t b = level_out[v] == FPO_NONE ? max_level + 1 : level_out[v];
        cnt[b + 1]++;
    }
    for (uint32_t b = 0; b <= max_level + 1; ++b) cnt[b + 1] += cnt[b];
    for (uint32_t v = 0; v < V; ++v) {
        uint32_t b = level_out[v] == FPO_NONE ? max_level + 1 : level_out[v];
        order_out[cnt[b]++] = v;
    }
    free(cnt); free(queue); free(indeg);
    return n_cycle;
}

/* ------------------------------------------------------------------------- */
/* A6  SPEC.md 2.3: FFD key (cpu desc, mem desc, index asc).                  */
/* ------------------------------------------------------------------------- */
/* thread-local: the bench CPU baseline and tests run the oracle on many host threads */
static _Thread_local const uint32_t *g_cpu, *g_mem;
static int ffd_cmp(const void *a, const void *b) {
    uint32_t i = *(const uint32_t *)a, j = *(const uint32_t *)b;
    if (g_cpu[i] != g_cpu[j]) return g_cpu[i] > g_cpu[j] ? -1 : 1;
    if (g_mem[i] != g_mem[j]) return g_mem[i] > g_mem[j] ? -1 : 1;
    return i < j ? -1 : (i > j ? 1 : 0);
}
void fpo_ffd_order(uint32_t C, const uint32_t *cpu_m, const uint32_t *mem_mib, uint32_t *order_out) {
    for (uint32_t i = 0; i < C; ++i) order_out[i] = i;
    g_cpu = cpu_m; g_mem = mem_mib;
    qsort(order_out, C, sizeof(uint32_t), ffd_cmp);
}

static inline int node_fits(uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf,
                            uint32_t cf, uint32_t mf, uint32_t lab, uint32_t cu, uint8_t sched) {
    return sched && cf >= cpu && mf >= mem && (lab & req) == req && (cu & conf) == 0;
}

/* A6 first fit on the lowest node index.  N == 1 with unconstrained capacity is
 * exactly controlplane/src/handlers/deploy.rs:390-394 (`servers.first()`). */
uint32_t fpo_place(uint32_t C, const uint32_t *cpu_m, const uint32_t *mem_mib,
                   const uint32_t *req_labels, const uint32_t *conflict,
                   uint32_t N, uint32_t *cpu_free, uint32_t *mem_free,
                   const uint32_t *labels, uint32_t *conflict_used, const uint8_t *schedulable,
                   const uint32_t *level, uint32_t *assign_out, uint8_t *reason_out,
                   uint64_t *evals_out) {
    uint32_t *order = (uint32_t *)malloc((C ? C : 1) * sizeof(uint32_t));
    fpo_ffd_order(C, cpu_m, mem_mib, order);
    uint32_t rejected = 0;
    uint64_t evals = 0;
    for (uint32_t k = 0; k < C; ++k) {
        uint32_t c = order[k];
        if (level && level[c] == FPO_NONE) {
            assign_out[c] = FPO_NONE; reason_out[c] = FPO_CYCLE; rejected++;
            continue;
        }
        uint32_t hit = FPO_NONE;
        for (uint32_t n = 0; n < N; ++n) {
            evals++;
            if (node_fits(cpu_m[c], mem_mib[c], req_labels[c], conflict[c],
                          cpu_free[n], mem_free[n], labels[n], conflict_used[n], schedulable[n])) {
                hit = n;
                break;
            }
        }
        if (hit == FPO_NONE) {
            assign_out[c] = FPO_NONE; reason_out[c] = FPO_NOFIT; rejected++;
        } else {
            cpu_free[hit] -= cpu_m[c];
            mem_free[hit] -= mem_mib[c];
            conflict_used[hit] |= conflict[c];
            assign_out[c] = hit; reason_out[c] = FPO_OK;
        }
    }
    free(order);
    if (evals_out) *evals_out = evals;
    return rejected;
}

void fpo_feasibility(uint32_t C, const uint32_t *cpu_m, const uint32_t *mem_mib,
                     const uint32_t *req_labels, const uint32_t *conflict,
                     uint32_t N, const uint32_t *cpu_free, const uint32_t *mem_free,
                     const uint32_t *labels, const uint32_t *conflict_used, const uint8_t *schedulable,
                     uint32_t *first_out, uint32_t *count_out, uint64_t *bitmap_out) {
    uint32_t WC = (C + 63) / 64;
    if (bitmap_out) memset(bitmap_out, 0, (size_t)WC * N * sizeof(uint64_t));
    for (uint32_t c = 0; c < C; ++c) {
        uint32_t first = FPO_NONE, cnt = 0;
        for (uint32_t n = 0; n < N; ++n) {
            if (node_fits(cpu_m[c], mem_mib[c], req_labels[c], conflict[c],
                          cpu_free[n], mem_free[n], labels[n], conflict_used[n], schedulable[n])) {
                if (first == FPO_NONE) first = n;
                cnt++;
                if (bitmap_out) bitmap_out[(size_t)(c / 64) * N + n] |= 1ull << (c % 64);
            }
        }
        first_out[c] = first;
        count_out[c] = cnt;
    }
}

/* SPEC.md 2.4 / SURVEY 8(e): lower is better; lowest scenario id wins ties. */
uint64_t fpo_cost(uint32_t C, const uint32_t *assign, uint32_t N, uint32_t scenario_id) {
    uint8_t *used = (uint8_t *)calloc(N ? N : 1, 1);
    uint64_t rej = 0, nused = 0;
    for (uint32_t c = 0; c < C; ++c) {
        if (assign[c] == FPO_NONE) rej++;
        else if (!used[assign[c]]) { used[assign[c]] = 1; nused++; }
    }
    free(used);
    if (rej > 0xFFFFFF) rej = 0xFFFFFF;
    if (nused > 0xFFFFFF) nused = 0xFFFFFF;
    return (rej << 40) | (nused << 16) | (scenario_id & 0xFFFFu);
}

/* ------------------------------------------------------------------------- */
/* SPEC.md 3: SplitMix64 in counter form: draw(seed, k) is the (k+1)-th       */
/* output of a SplitMix64 generator whose state starts at `seed`.             */
/* ------------------------------------------------------------------------- */
#define GAMMA 0x9E3779B97F4A7C15ull
#define TAG_CONT 0xC0C0C0C0C0C0C0C0ull
#define TAG_NODE 0x5E5E5E5E5E5E5E5Eull
#define TAG_DAG 0xDADADADADADADADAull

uint64_t fpo_splitmix_draw(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * GAMMA;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t fpo_scenario_seed(uint64_t seed, uint32_t scenario) {
    return seed ^ ((uint64_t)scenario * GAMMA);
}

void fpo_gen_containers(uint64_t seed, uint32_t C, uint32_t flags,
                        uint32_t *cpu_m, uint32_t *mem_mib, uint32_t *req_labels, uint32_t *conflict) {
    uint64_t s = seed ^ TAG_CONT;
    for (uint32_t j = 0; j < C; ++j) {
        uint64_t k = (uint64_t)j * 8;
        cpu_m[j] = 50u * (2u + (uint32_t)(fpo_splitmix_draw(s, k + 0) % 79u));
        mem_mib[j] = 64u * (1u + (uint32_t)(fpo_splitmix_draw(s, k + 1) % 256u));
        uint32_t cf = 0, rq = 0;
        if ((flags & 1u) && fpo_splitmix_draw(s, k + 2) % 1000u < 100u)
            cf |= 1u << (fpo_splitmix_draw(s, k + 3) % 16u);
        if ((flags & 2u) && fpo_splitmix_draw(s, k + 4) % 1000u < 200u)
            cf |= 1u << (16u + fpo_splitmix_draw(s, k + 5) % 16u);
        if ((flags & 4u) && fpo_splitmix_draw(s, k + 6) % 1000u < 300u)
            rq = 1u << (fpo_splitmix_draw(s, k + 7) % 13u);
        conflict[j] = cf;
        req_labels[j] = rq;
    }
}

void fpo_gen_nodes(uint64_t seed, uint32_t N, uint32_t flags,
                   uint32_t *cpu_free, uint32_t *mem_free, uint32_t *labels,
                   uint32_t *conflict_used, uint8_t *schedulable) {
    static const uint32_t CPU[5] = {4000, 8000, 16000, 32000, 64000};
    static const uint32_t MEM[5] = {8192, 16384, 32768, 65536, 262144};
    uint64_t s = seed ^ TAG_NODE;
    (void)flags;
    for (uint32_t n = 0; n < N; ++n) {
        uint64_t k = (uint64_t)n * 8;
        uint32_t t = (uint32_t)(fpo_splitmix_draw(s, k + 0) % 5u);
        cpu_free[n] = CPU[t];
        mem_free[n] = MEM[t];
        uint32_t lab = 0;
        lab |= 1u << (0u + fpo_splitmix_draw(s, k + 1) % 3u);  /* tier   bits 0-2  */
        lab |= 1u << (3u + fpo_splitmix_draw(s, k + 2) % 4u);  /* region bits 3-6  */
        lab |= 1u << (7u + fpo_splitmix_draw(s, k + 3) % 4u);  /* class  bits 7-10 */
        lab |= 1u << (11u + fpo_splitmix_draw(s, k + 4) % 2u); /* arch   bits 11-12 */
        labels[n] = lab;
        conflict_used[n] = 0;
        schedulable[n] = (fpo_splitmix_draw(s, k + 5) % 1000u) >= 20u ? 1 : 0;
    }
}

/* SPEC.md 3.3: config-5 DAG. */
uint32_t fpo_dag_vertices(uint32_t n_chains, uint32_t chain_len, uint32_t n_layers, uint32_t layer_width) {
    return n_chains * chain_len + n_layers * layer_width;
}

typedef struct { uint32_t dep, dependent; } edge_t;

static uint32_t dag_edges(uint64_t seed, uint32_t n_chains, uint32_t chain_len,
                          uint32_t n_layers, uint32_t layer_width, uint32_t n_cycles,
                          edge_t *out /* may be NULL */) {
    uint64_t s = seed ^ TAG_DAG;
    uint32_t n_chain_v = n_chains * chain_len;
    uint32_t E = 0;
    for (uint32_t k = 0; k < n_chains; ++k)
        for (uint32_t i = 1; i < chain_len; ++i) {
            if (out) { out[E].dep = k * chain_len + i - 1; out[E].dependent = k * chain_len + i; }
            E++;
        }
    for (uint32_t L = 0; L < n_layers; ++L) {
        uint32_t pool = n_chain_v + L * layer_width;
        for (uint32_t j = 0; j < layer_width; ++j) {
            uint32_t v = n_chain_v + L * layer_width + j;
            uint64_t k = (uint64_t)v * 8;
            uint32_t m = pool ? 1u + (uint32_t)(fpo_splitmix_draw(s, k) % 4u) : 0u;
            for (uint32_t q = 0; q < m; ++q) {
                if (out) {
                    out[E].dep = (uint32_t)(fpo_splitmix_draw(s, k + 1 + q) % pool);
                    out[E].dependent = v;
                }
                E++;
            }
        }
    }
    /* 3-cycles among the last layer's vertices: a->b->c->a in depends_on terms */
    if (n_layers > 0 && layer_width >= 3) {
        uint32_t base = n_chain_v + (n_layers - 1) * layer_width;
        for (uint32_t q = 0; q < n_cycles && 3 * q + 2 < layer_width; ++q) {
            uint32_t a = base + 3 * q, b = a + 1, c = a + 2;
            if (out) {
                out[E + 0].dep = b; out[E + 0].dependent = a;
                out[E + 1].dep = c; out[E + 1].dependent = b;
                out[E + 2].dep = a; out[E + 2].dependent = c;
            }
            E += 3;
        }
    }
    return E;
}

/* Vertex ids are the logical ids pushed through a Fisher-Yates permutation. */
static void dag_perm(uint64_t seed, uint32_t V, uint32_t *perm) {
    uint64_t s = seed ^ TAG_DAG ^ 0x1111111111111111ull;
    for (uint32_t i = 0; i < V; ++i) perm[i] = i;
    for (uint32_t i = V; i > 1; --i) {
        uint32_t j = (uint32_t)(fpo_splitmix_draw(s, i) % i);
        uint32_t t = perm[i - 1]; perm[i - 1] = perm[j]; perm[j] = t;
    }
}

uint32_t fpo_gen_dag(uint64_t seed, uint32_t n_chains, uint32_t chain_len,
                     uint32_t n_layers, uint32_t layer_width, uint32_t n_cycles,
                     uint32_t *row_ptr, uint32_t *col, uint8_t *has_deps) {
    uint32_t V = fpo_dag_vertices(n_chains, chain_len, n_layers, layer_width);
    uint32_t E = dag_edges(seed, n_chains, chain_len, n_layers, layer_width, n_cycles, NULL);
    edge_t *ed = (edge_t *)malloc((E ? E : 1) * sizeof(edge_t));
    uint32_t *perm = (uint32_t *)malloc((V ? V : 1) * sizeof(uint32_t));
    dag_edges(seed, n_chains, chain_len, n_layers, layer_width, n_cycles, ed);
    dag_perm(seed, V, perm);
    memset(row_ptr, 0, ((size_t)V + 1) * sizeof(uint32_t));
    memset(has_deps, 0, V);
    for (uint32_t e = 0; e < E; ++e) {
        row_ptr[perm[ed[e].dep] + 1]++;
        has_deps[perm[ed[e].dependent]] = 1;
    }
    for (uint32_t v = 0; v < V; ++v) row_ptr[v + 1] += row_ptr[v];
    if (col) {
        uint32_t *fill = (uint32_t *)malloc((V ? V : 1) * sizeof(uint32_t));
        memcpy(fill, row_ptr, V * sizeof(uint32_t));
        for (uint32_t e = 0; e < E; ++e) col[fill[perm[ed[e].dep]]++] = perm[ed[e].dependent];
        free(fill);
    }
    free(perm); free(ed);
    return E;
}
