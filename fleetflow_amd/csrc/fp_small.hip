// fp_small.hip -- a whole stage plan in one launch (fp_plan_stage, include/fleetplace.h).
//
// The `fleet up --dry-run` path (crates/fleetflow/src/commands/up.rs:57-136) plans one stage of a
// fleet.kdl: a handful of services and servers (BASELINE config 1).  Planned as separate
// host-pointer calls -- fp_legacy_order, fp_levelize, fp_feasibility, fp_place -- each pays its
// own copies in, launch, copy back and synchronisation (~70 us per plan in round 4).  Here a stage
// of at most LS_V services, LS_E edges and SMALL_MAX_N servers is ONE kernel, k_plan_small, that
// reads its inputs from and writes its results to mapped pinned host memory: one launch and one
// stream synchronisation per plan, no copy calls.  In one workgroup's LDS it computes
//   * A1 the legacy start order (engine.rs:67-85: has_deps == 0 first, each part in input order);
//   * A2 Kahn levels and the (level, index) start order (fps::ls_levels, SPEC.md 2.2);
//   * with servers: stage 2 on the pristine table (feasible-server count and first feasible server
//     per service, SPEC.md 2.5: the dry-run candidates) and A6 first-fit-decreasing (SPEC.md 2.3)
//     with the levels' CYCLE gate, the node table updated in place.
// Larger stages run the general kernels through the same host calls as before.
#include "fp_internal.h"
#include <chrono>
#include "fp_small.h"
#include <string.h>
#include <vector>

namespace {

constexpr uint32_t SMALL_MAX_N = 4096;
constexpr size_t SMALL_LDS_CAP = 160 * 1024;

struct PlanSmallArgs {
    // inputs (mapped host memory)
    const uint32_t *rp, *col;
    const uint8_t *hd;
    const uint32_t *cpu, *mem, *req, *conf;  // [V] (container v = vertex v); place only
    const uint32_t *cf, *mf, *lab, *cu;      // [N]; place only
    const uint8_t *sched;
    uint32_t V, E, N, place;
    // outputs (mapped host memory)
    uint32_t *perm, *level, *order, *ncyc, *err;
    uint32_t *first, *count, *assign;  // [V]; place only
    uint8_t *reason;
    uint32_t *cf_out, *mf_out, *cu_out;  // [N]; place only
};

__host__ __device__ inline size_t words4(size_t bytes) { return (bytes + 15) / 16 * 4; }  // 16-B aligned words

// LDS words of k_plan_small for a stage of V services, E edges and N servers
inline size_t plan_small_words(uint32_t V, uint32_t E, uint32_t N, bool place) {
    size_t w = words4((size_t)(V + 1) * 4) + words4((size_t)E * 4) + words4(V) + words4(fps::ls_words(V) * 4) +
               2 * words4((size_t)V * 4);
    if (place) w += 4 * words4((size_t)V * 4) + 4 * words4((size_t)N * 4) + words4(N) + words4((size_t)V * 4);
    return w;
}

// The completion word of k_plan_small: written last, with system-scope release, in mapped host
// memory; fp_plan_stage polls it instead of synchronising the stream
__device__ __forceinline__ void plan_small_done(uint32_t *err, uint32_t v) {
    __hip_atomic_store(err, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void k_plan_small(const PlanSmallArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    __shared__ uint32_t wsum[16];
    const uint32_t V = a.V, E = a.E, N = a.N, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t nw = blockDim.x >> 6;
    uint32_t *rp = sm;
    uint32_t *col = rp + words4((size_t)(V + 1) * 4);
    uint8_t *hd = (uint8_t *)(col + words4((size_t)E * 4));
    uint32_t *ks = (uint32_t *)hd + words4(V);
    uint32_t *lv = ks + words4(fps::ls_words(V) * 4);
    uint32_t *od = lv + words4((size_t)V * 4);
    uint32_t *cpu = od + words4((size_t)V * 4), *mem = cpu + words4((size_t)V * 4);
    uint32_t *req = mem + words4((size_t)V * 4), *conf = req + words4((size_t)V * 4);
    uint32_t *cf = conf + words4((size_t)V * 4), *mf = cf + words4((size_t)N * 4);
    uint32_t *lab = mf + words4((size_t)N * 4), *cu = lab + words4((size_t)N * 4);
    uint8_t *sch = (uint8_t *)(cu + words4((size_t)N * 4));
    uint32_t *srt = (uint32_t *)sch + words4(N);

    // inputs -> LDS: every load of a pass in flight at once (PCIe round trips, not bandwidth)
    for (uint32_t i = t; i <= V; i += blockDim.x) rp[i] = a.rp[i];
    for (uint32_t i = t; i < E; i += blockDim.x) col[i] = a.col[i];
    for (uint32_t i = t; i < V; i += blockDim.x) hd[i] = a.hd[i];
    if (a.place) {
        for (uint32_t i = t; i < V; i += blockDim.x) {
            cpu[i] = a.cpu[i];
            mem[i] = a.mem[i];
            req[i] = a.req[i];
            conf[i] = a.conf[i];
        }
        for (uint32_t i = t; i < N; i += blockDim.x) {
            cf[i] = a.cf[i];
            mf[i] = a.mf[i];
            lab[i] = a.lab[i];
            cu[i] = a.cu[i];
            sch[i] = a.sched[i];
        }
    }
    __syncthreads();

    // A2: levels and the start order (the CSR check first: a corrupt CSR writes nothing else)
    const uint32_t nc = fps::ls_levels(rp, col, hd, V, E, ks, lv, od);
    if (nc == FP_NONE) {
        if (t == 0) plan_small_done(a.err, (uint32_t)(-FP_ECORRUPT));
        return;  // uniform
    }

    // A1: stable partition, has_deps == 0 first (V <= LS_V <= blockDim: one vertex per thread)
    {
        const bool z = t < V && hd[t] == 0;
        const uint64_t m = __builtin_amdgcn_ballot_w64(z);
        if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t woff = 0, tot = 0;
        for (uint32_t q = 0; q < nw; ++q) {
            woff += q < w ? wsum[q] : 0u;
            tot += wsum[q];
        }
        if (t < V) {
            const uint32_t zb = woff + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));  // zeros before t
            a.perm[z ? zb : tot + t - zb] = t;
        }
    }
    for (uint32_t i = t; i < V; i += blockDim.x) {
        a.level[i] = lv[i];
        a.order[i] = od[i];
    }
    if (t == 0) *a.ncyc = nc;

    if (a.place) {
        // stage 2 on the pristine table (SPEC.md 2.5): wave w takes services w, w + nw, ...; lanes
        // are servers
        for (uint32_t v = w; v < V; v += nw) {
            const uint32_t c = cpu[v], m = mem[v], r = req[v], x = conf[v];
            uint32_t cnt = 0, first = FP_NONE;
            for (uint32_t n0 = 0; n0 < N; n0 += 64) {
                const uint32_t n = n0 + lane;
                const bool f = n < N && sch[n] && fpd::fits(c, m, r, x, cf[n], mf[n], lab[n], cu[n]);
                const uint64_t b = __builtin_amdgcn_ballot_w64(f);
                cnt += (uint32_t)__popcll(b);
                if (first == FP_NONE && b) first = n0 + (uint32_t)__builtin_ctzll(b);
            }
            if (lane == 0) {
                a.first[v] = first;
                a.count[v] = cnt;
            }
        }
        // FFD order (SPEC.md 2.3 step 1): the rank of service v under (cpu desc, mem desc, index asc)
        for (uint32_t v = t; v < V; v += blockDim.x) {
            const uint32_t c = cpu[v], m = mem[v];
            uint32_t r = 0;
            for (uint32_t u = 0; u < V; ++u) {
                const uint32_t cu_ = cpu[u], mu = mem[u];
                r += (cu_ > c || (cu_ == c && (mu > m || (mu == m && u < v)))) ? 1u : 0u;
            }
            srt[r] = v;
        }
        __syncthreads();  // the candidates read the pristine table; the fill below changes it
        // sequential first fit by wave 0 (SPEC.md 2.3 step 2): lanes test 64 servers at a time, the
        // lowest fitting lane takes the service
        if (w == 0) {
            for (uint32_t k = 0; k < V; ++k) {
                const uint32_t v = srt[k];
                uint32_t asg = FP_NONE, rs = FP_REASON_NOFIT;
                if (lv[v] == FP_NONE) {
                    rs = FP_REASON_CYCLE;
                } else {
                    const uint32_t c = cpu[v], m = mem[v], r = req[v], x = conf[v];
                    for (uint32_t n0 = 0; n0 < N; n0 += 64) {
                        const uint32_t n = n0 + lane;
                        const bool f = n < N && sch[n] && fpd::fits(c, m, r, x, cf[n], mf[n], lab[n], cu[n]);
                        const uint64_t b = __builtin_amdgcn_ballot_w64(f);
                        if (b) {  // uniform
                            const uint32_t l = (uint32_t)__builtin_ctzll(b);
                            if (lane == l) {
                                cf[n] -= c;
                                mf[n] -= m;
                                cu[n] |= x;
                            }
                            asg = n0 + l;
                            rs = FP_REASON_OK;
                            break;
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the update before the next test
                }
                if (lane == 0) {
                    a.assign[v] = asg;
                    a.reason[v] = (uint8_t)rs;
                }
            }
        }
        __syncthreads();
        for (uint32_t i = t; i < N; i += blockDim.x) {
            a.cf_out[i] = cf[i];
            a.mf_out[i] = mf[i];
            a.cu_out[i] = cu[i];
        }
    }
    // every thread's results reach host memory before the completion word (the host polls it)
    __threadfence_system();
    __syncthreads();
    if (t == 0) plan_small_done(a.err, 0u);
}

// ---- stages of at most 64 services: one wave, inputs in the kernel arguments ----
// A fleet.kdl stage holds a handful of services (config 1: 2-3).  k_plan_small above reads its
// inputs from mapped host memory in dependent passes and synchronises 16 waves between phases
// (9.4 us of kernel time for 3 services, r06s).  k_plan_tiny takes the whole stage by value in its
// kernel arguments (the launch copies them into the dispatch's kernarg buffer), computes with one
// wave -- lane v = service v, lane n = server n -- and writes one tagged word per service to
// mapped host memory, which the host polls: no host-memory reads, no barriers, no completion flag.
constexpr uint32_t TINY_V = 64, TINY_E = 256, TINY_N = 64;

struct PlanTinyArgs {
    uint32_t V, E, N, tag;
    uint64_t *out;     // [V] tagged service words (mapped host memory)
    uint32_t *nodes;   // [3][N] cpu_free / mem_free / conflict_used after the fill (place only)
    uint16_t rp[TINY_V + 1];  // row_ptr, clamped to 0xFFFF (a larger value is corrupt anyway)
    uint8_t col[TINY_E];      // col, clamped to 0xFF (>= V: corrupt)
    uint8_t hd[TINY_V];
};
struct PlanTinyPlaceArgs {
    PlanTinyArgs g;
    uint32_t cpu[TINY_V], mem[TINY_V], req[TINY_V], conf[TINY_V];
    uint32_t cf[TINY_N], mf[TINY_N], lab[TINY_N], cu[TINY_N];
    uint64_t sched;  // bit n: server n schedulable
};
static_assert(sizeof(PlanTinyPlaceArgs) <= 4096, "kernel arguments are at most 4 KB");

// the service word: perm | order << 8 | level << 16 (0xFF: CYCLE) | first << 24 (0xFF: none) |
// count << 32 | assign << 40 (0xFF: none) | reason << 48 | tag << 56; a corrupt CSR writes 0xFF in
// the perm byte of every word (perm < V <= 64 otherwise)
constexpr uint64_t TINY_CORRUPT = 0xFFull;

// the body of both kernels: `a` is read through the kernarg pointer (lane-indexed fields are plain
// loads from the dispatch's argument buffer, uniform ones scalar loads); PLACE reads the place part
template <bool PLACE>
__device__ __forceinline__ void plan_tiny_body(const PlanTinyPlaceArgs &a) {
    __shared__ uint64_t par[TINY_V];  // parent set of each vertex
    const uint32_t lane = threadIdx.x, V = a.g.V, E = a.g.E, N = a.g.N;
    const uint64_t tagw = (uint64_t)a.g.tag << 56;
    const bool valid = lane < V;
    // CSR check (k_check_csr's conditions) and the parent sets
    const uint32_t r0 = valid ? a.g.rp[lane] : 0u, r1 = valid ? a.g.rp[lane + 1] : 0u;
    bool bad = valid && r1 < r0;
    for (uint32_t e = lane; e < E; e += 64) bad |= a.g.col[e] >= V;
    bad |= a.g.rp[0] != 0u || a.g.rp[V] != E;
    par[lane] = 0ull;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (__builtin_amdgcn_ballot_w64(bad)) {
        if (valid) a.g.out[lane] = tagw | TINY_CORRUPT;
        return;
    }
    if (valid)
        for (uint32_t e = r0; e < r1; ++e) atomicOr(&par[a.g.col[e]], 1ull << lane);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint64_t pm = par[lane];
    // Kahn levels (SPEC.md 2.2): a vertex is ready once its parents are done; its level is
    // max(has_deps ? 1 : 0, parents' levels + 1), pushed by each parent when it is done
    uint32_t lvl = valid && a.g.hd[lane] ? 1u : 0u;
    uint64_t done = 0;
    while (true) {
        const uint64_t ready = __builtin_amdgcn_ballot_w64(valid && !((done >> lane) & 1ull) && (pm & ~done) == 0ull);
        if (!ready) break;
        for (uint64_t r = ready; r;) {
            const uint32_t u = (uint32_t)__builtin_ctzll(r);
            r &= r - 1;
            const uint32_t lu = (uint32_t)__builtin_amdgcn_readlane((int)lvl, (int)u) + 1u;
            lvl = ((pm >> u) & 1ull) && lu > lvl ? lu : lvl;
        }
        done |= ready;
    }
    const bool cyc = valid && !((done >> lane) & 1ull);
    uint32_t maxl = !cyc && valid ? lvl : 0u;
    for (int o = 32; o; o >>= 1) maxl = max(maxl, (uint32_t)__shfl_xor((int)maxl, o));
    const uint32_t ck = (maxl > 1u ? maxl : 1u) + 1u;
    // start order: stable by (level, index), CYCLE last -- rank by a bitwise comparison of the keys
    const uint32_t key = cyc ? ck : lvl;
    uint64_t eq = __builtin_amdgcn_ballot_w64(valid), lt = 0;
    for (int b = 6; b >= 0; --b) {  // keys <= 65
        const uint64_t B = __builtin_amdgcn_ballot_w64(valid && ((key >> b) & 1u));
        if ((key >> b) & 1u) { lt |= eq & ~B; eq &= B; }
        else eq &= ~B;
    }
    const uint64_t below = (1ull << lane) - 1ull;
    // (lanes past V take their own index: ds_permute destinations stay distinct)
    const uint32_t rank = valid ? (uint32_t)__popcll(lt) + (uint32_t)__popcll(eq & below) : lane;
    const uint32_t ord = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank << 2), (int)lane);
    // A1 legacy order (engine.rs:67-85): has_deps == 0 first, each part in input order
    const uint64_t zm = __builtin_amdgcn_ballot_w64(valid && a.g.hd[lane] == 0);
    const uint32_t zb = (uint32_t)__popcll(zm & below), tot = (uint32_t)__popcll(zm);
    const uint32_t ppos = (zm >> lane) & 1ull ? zb : tot + lane - zb;
    const uint32_t perm = (uint32_t)__builtin_amdgcn_ds_permute((int)(ppos << 2), (int)lane);
    uint64_t w = tagw | perm | ((uint64_t)ord << 8) | ((uint64_t)(cyc ? 0xFFu : lvl) << 16);
    if (PLACE) {
        const uint32_t c = valid ? a.cpu[lane] : 0u, m = valid ? a.mem[lane] : 0u;
        const uint32_t r = valid ? a.req[lane] : 0u, x = valid ? a.conf[lane] : 0u;
        // stage 2 on the pristine table (SPEC.md 2.5): feasible servers and the first one
        uint32_t cnt = 0, first = 0xFFu;
        for (uint32_t n = 0; n < N; ++n) {
            const bool f = ((a.sched >> n) & 1ull) && fpd::fits(c, m, r, x, a.cf[n], a.mf[n], a.lab[n], a.cu[n]);
            cnt += f ? 1u : 0u;
            first = f && first == 0xFFu ? n : first;
        }
        // FFD order (SPEC.md 2.3 step 1): rank under (cpu desc, mem desc, index asc)
        uint32_t fr = 0;
        for (uint32_t u = 0; u < V; ++u) {
            const uint32_t cu_ = a.cpu[u], mu = a.mem[u];
            fr += (cu_ > c || (cu_ == c && (mu > m || (mu == m && u < lane)))) ? 1u : 0u;
        }
        fr = valid ? fr : lane;
        const uint32_t srt = (uint32_t)__builtin_amdgcn_ds_permute((int)(fr << 2), (int)lane);
        // sequential first fit: lanes = servers, the node state in registers
        const bool live = lane < N && ((a.sched >> lane) & 1ull);
        uint32_t ncf = lane < N ? a.cf[lane] : 0u, nmf = lane < N ? a.mf[lane] : 0u;
        uint32_t ncu = lane < N ? a.cu[lane] : 0u;
        const uint32_t nlab = lane < N ? a.lab[lane] : 0u;
        uint32_t asg = 0xFFu, rsn = FP_REASON_NOFIT;
        for (uint32_t k = 0; k < V; ++k) {
            const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)srt, (int)k);
            uint32_t to = 0xFFu, rs = FP_REASON_NOFIT;
            if ((done >> v) & 1ull) {  // not a CYCLE member
                const uint32_t vc = a.cpu[v], vm = a.mem[v], vr = a.req[v], vx = a.conf[v];
                const uint64_t fit = __builtin_amdgcn_ballot_w64(live && fpd::fits(vc, vm, vr, vx, ncf, nmf, nlab, ncu));
                if (fit) {
                    const uint32_t l = (uint32_t)__builtin_ctzll(fit);
                    if (lane == l) { ncf -= vc; nmf -= vm; ncu |= vx; }
                    to = l;
                    rs = FP_REASON_OK;
                }
            } else {
                rs = FP_REASON_CYCLE;
            }
            asg = lane == v ? to : asg;
            rsn = lane == v ? rs : rsn;
        }
        if (lane < N) {
            a.g.nodes[lane] = ncf;
            a.g.nodes[TINY_N + lane] = nmf;
            a.g.nodes[2 * TINY_N + lane] = ncu;
        }
        __threadfence_system();  // the node state lands before the tagged words the host polls
        w |= ((uint64_t)first << 24) | ((uint64_t)cnt << 32) | ((uint64_t)asg << 40) | ((uint64_t)rsn << 48);
    }
    if (valid) a.g.out[lane] = w;
}

// the stage without servers (the config-1 fixtures): only the graph part as arguments
__global__ __launch_bounds__(64) void k_plan_tiny(const PlanTinyArgs a_arg) {
#if defined(__HIP_DEVICE_COMPILE__)
    plan_tiny_body<false>(*(const PlanTinyPlaceArgs *)__builtin_amdgcn_kernarg_segment_ptr());
#else
    (void)a_arg;
#endif
}
__global__ __launch_bounds__(64) void k_plan_tiny_place(const PlanTinyPlaceArgs a_arg) {
#if defined(__HIP_DEVICE_COMPILE__)
    plan_tiny_body<true>(*(const PlanTinyPlaceArgs *)__builtin_amdgcn_kernarg_segment_ptr());
#else
    (void)a_arg;
#endif
}

// the general path: the separate host-pointer calls into temporaries, committed only when all
// succeeded (on error nothing is written)
int plan_general(fp_ctx *c, const fp_graph *g, const fp_containers *cs, fp_nodes *ns, uint32_t *perm_out,
                 uint32_t *level_out, uint32_t *order_out, uint32_t *n_cycle_out, uint32_t *first_out,
                 uint32_t *count_out, uint32_t *assign_out, uint8_t *reason_out) {
    const size_t V = g->n_vertices, N = ns ? ns->n : 0;
    std::vector<uint32_t> perm(V), lev(V), ord(V), first(ns ? V : 0), count(ns ? V : 0), asg(ns ? V : 0);
    std::vector<uint8_t> rsn(ns ? V : 0);
    std::vector<uint32_t> cf, mf, cu;
    uint32_t nc = 0;
    int rc = fp_legacy_order(c, g, perm.data());
    if (!rc) rc = fp_levelize(c, g, lev.data(), ord.data(), &nc);
    if (!rc && ns) {
        rc = fp_feasibility(c, cs, ns, first.data(), count.data(), nullptr);
        if (!rc) {
            cf.assign(ns->cpu_free, ns->cpu_free + N);
            mf.assign(ns->mem_free, ns->mem_free + N);
            cu.assign(ns->conflict_used, ns->conflict_used + N);
            fp_nodes tn = *ns;
            tn.cpu_free = cf.data();
            tn.mem_free = mf.data();
            tn.conflict_used = cu.data();
            rc = fp_place(c, cs, &tn, lev.data(), asg.data(), rsn.data());
        }
    }
    if (rc) return rc;
    memcpy(perm_out, perm.data(), V * 4);
    memcpy(level_out, lev.data(), V * 4);
    memcpy(order_out, ord.data(), V * 4);
    if (n_cycle_out) *n_cycle_out = nc;
    if (ns) {
        if (first_out) memcpy(first_out, first.data(), V * 4);
        if (count_out) memcpy(count_out, count.data(), V * 4);
        memcpy(assign_out, asg.data(), V * 4);
        memcpy(reason_out, rsn.data(), V);
        memcpy(ns->cpu_free, cf.data(), N * 4);
        memcpy(ns->mem_free, mf.data(), N * 4);
        memcpy(ns->conflict_used, cu.data(), N * 4);
    }
    return FP_OK;
}

// fp_plan_stage for V <= TINY_V, E <= TINY_E, N <= TINY_N (arguments checked by the caller)
int plan_tiny(fp_ctx *c, const fp_graph *g, const fp_containers *cs, fp_nodes *ns, uint32_t *perm_out,
              uint32_t *level_out, uint32_t *order_out, uint32_t *n_cycle_out, uint32_t *first_out,
              uint32_t *count_out, uint32_t *assign_out, uint8_t *reason_out) {
    const uint32_t V = g->n_vertices, E = g->n_edges, N = ns ? ns->n : 0;
    const bool place = ns != nullptr;
    FP_HIP(hipSetDevice(c->device));
    if (!c->h_tiny) {
        FP_HIP(hipHostMalloc((void **)&c->h_tiny, 4096, hipHostMallocMapped | hipHostMallocCoherent));
        FP_HIP(hipHostGetDevicePointer(&c->d_tiny, c->h_tiny, 0));
        memset(c->h_tiny, 0, 4096);
    }
    volatile uint64_t *hw = (volatile uint64_t *)c->h_tiny;
    const uint32_t *hn = (const uint32_t *)(c->h_tiny + TINY_V * 8);
    c->tiny_tag = c->tiny_tag % 255u + 1u;  // 1..255; the words polled below are zeroed first
    const uint32_t tag = c->tiny_tag;
    for (uint32_t v = 0; v < V; ++v) hw[v] = 0ull;
    PlanTinyPlaceArgs a;
    a.g.V = V; a.g.E = E; a.g.N = N; a.g.tag = tag;
    a.g.out = (uint64_t *)c->d_tiny;
    a.g.nodes = (uint32_t *)((char *)c->d_tiny + TINY_V * 8);
    for (uint32_t i = 0; i <= V; ++i) a.g.rp[i] = (uint16_t)(g->row_ptr[i] < 0xFFFFu ? g->row_ptr[i] : 0xFFFFu);
    for (uint32_t e = 0; e < E; ++e) a.g.col[e] = (uint8_t)(g->col[e] < 0xFFu ? g->col[e] : 0xFFu);
    memcpy(a.g.hd, g->has_deps, V);
    if (place) {
        memcpy(a.cpu, cs->cpu_m, V * 4); memcpy(a.mem, cs->mem_mib, V * 4);
        memcpy(a.req, cs->req_labels, V * 4); memcpy(a.conf, cs->conflict, V * 4);
        a.sched = 0;
        for (uint32_t n = 0; n < N; ++n) {
            a.cf[n] = ns->cpu_free[n]; a.mf[n] = ns->mem_free[n]; a.lab[n] = ns->labels[n]; a.cu[n] = ns->conflict_used[n];
            a.sched |= ns->schedulable[n] ? 1ull << n : 0ull;
        }
    }
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_LEVEL, &ev);
    // the place-free kernel reads only the graph part of the arguments
    if (place) k_plan_tiny_place<<<1, 64, 0, c->stream>>>(a);
    else k_plan_tiny<<<1, 64, 0, c->stream>>>(a.g);
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_LEVEL, ev);
    // poll the tagged words (mapped, coherent host memory); the stream synchronisation is the
    // fallback for a kernel that has not finished after ~20 ms, and the path when profiling
    auto all_in = [&]() {
        for (uint32_t v = 0; v < V; ++v)
            if ((uint32_t)(__atomic_load_n(&hw[v], __ATOMIC_ACQUIRE) >> 56) != tag) return false;
        return true;
    };
    bool seen = false;
    if (!c->profile) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0;; ++spin) {
            if (all_in()) { seen = true; break; }
            if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
        }
    }
    if (!seen) {
        FP_HIP(hipStreamSynchronize(c->stream));
        if (!all_in()) return FP_EDEVICE;
    }
    if ((hw[0] & 0xFFull) == TINY_CORRUPT) return FP_ECORRUPT;
    uint32_t nc = 0;
    for (uint32_t v = 0; v < V; ++v) {
        const uint64_t x = hw[v];
        perm_out[v] = (uint32_t)(x & 0xFF);
        order_out[v] = (uint32_t)((x >> 8) & 0xFF);
        const uint32_t l = (uint32_t)((x >> 16) & 0xFF);
        level_out[v] = l == 0xFFu ? FP_NONE : l;
        nc += l == 0xFFu ? 1u : 0u;
        if (place) {
            const uint32_t f = (uint32_t)((x >> 24) & 0xFF), asg = (uint32_t)((x >> 40) & 0xFF);
            if (first_out) first_out[v] = f == 0xFFu ? FP_NONE : f;
            if (count_out) count_out[v] = (uint32_t)((x >> 32) & 0xFF);
            assign_out[v] = asg == 0xFFu ? FP_NONE : asg;
            reason_out[v] = (uint8_t)((x >> 48) & 0xFF);
        }
    }
    if (n_cycle_out) *n_cycle_out = nc;
    if (place && N) {
        memcpy(ns->cpu_free, hn, (size_t)N * 4);
        memcpy(ns->mem_free, hn + TINY_N, (size_t)N * 4);
        memcpy(ns->conflict_used, hn + 2 * TINY_N, (size_t)N * 4);
    }
    return FP_OK;
}

}  // namespace

extern "C" int fp_plan_stage(fp_ctx *c, const fp_graph *g, const fp_containers *cs, fp_nodes *ns,
                             uint32_t *perm_out, uint32_t *level_out, uint32_t *order_out, uint32_t *n_cycle_out,
                             uint32_t *first_out, uint32_t *count_out, uint32_t *assign_out, uint8_t *reason_out) {
    if (!c || !g) return FP_EINVAL;
    const uint32_t V = g->n_vertices, E = g->n_edges;
    const bool place = ns != nullptr;
    if (V && (!g->has_deps || !g->row_ptr || !perm_out || !level_out || !order_out)) return FP_EINVAL;
    if (E && !g->col) return FP_EINVAL;
    if (place) {
        if (!cs || cs->n != V) return FP_EINVAL;
        if (V && (!cs->cpu_m || !cs->mem_mib || !cs->req_labels || !cs->conflict || !assign_out || !reason_out))
            return FP_EINVAL;
        if (ns->n && (!ns->cpu_free || !ns->mem_free || !ns->labels || !ns->conflict_used || !ns->schedulable))
            return FP_EINVAL;
    }
    if (V == 0) {
        if (E) return FP_ECORRUPT;
        if (n_cycle_out) *n_cycle_out = 0;
        return FP_OK;
    }
    const uint32_t N = place ? ns->n : 0;
    // FP_OPT_LEVEL_SMALL: 0 = the general calls, 2 = k_plan_small without the one-wave path
    if (V <= TINY_V && E <= TINY_E && N <= TINY_N && fp_opt(c, FP_OPT_LEVEL_SMALL, 1) == 1)
        return plan_tiny(c, g, cs, ns, perm_out, level_out, order_out, n_cycle_out, first_out, count_out, assign_out,
                         reason_out);
    const size_t lds = plan_small_words(V, E, N, place) * 4;
    if (V > fps::LS_V || E > fps::LS_E || N > SMALL_MAX_N || lds > SMALL_LDS_CAP ||
        fp_opt(c, FP_OPT_LEVEL_SMALL, 1) == 0)
        return plan_general(c, g, cs, ns, perm_out, level_out, order_out, n_cycle_out, first_out, count_out,
                            assign_out, reason_out);
    FP_HIP(hipSetDevice(c->device));
    // packed mapped buffer: inputs, then outputs (u32 words, 16-B aligned regions)
    size_t off = 0;
    auto take = [&off](size_t bytes) { const size_t o = off; off += words4(bytes); return o; };
    const size_t i_rp = take((size_t)(V + 1) * 4), i_col = take((size_t)E * 4), i_hd = take(V);
    const size_t i_cpu = take(place ? (size_t)V * 4 : 0), i_mem = take(place ? (size_t)V * 4 : 0);
    const size_t i_req = take(place ? (size_t)V * 4 : 0), i_conf = take(place ? (size_t)V * 4 : 0);
    const size_t i_cf = take((size_t)N * 4), i_mf = take((size_t)N * 4), i_lab = take((size_t)N * 4);
    const size_t i_cu = take((size_t)N * 4), i_sch = take(N);
    const size_t o_perm = take((size_t)V * 4), o_lev = take((size_t)V * 4), o_ord = take((size_t)V * 4);
    const size_t o_ncyc = take(4), o_err = take(4);
    const size_t o_first = take(place ? (size_t)V * 4 : 0), o_count = take(place ? (size_t)V * 4 : 0);
    const size_t o_asg = take(place ? (size_t)V * 4 : 0), o_rsn = take(place ? V : 0);
    const size_t o_cf = take((size_t)N * 4), o_mf = take((size_t)N * 4), o_cu = take((size_t)N * 4);
    const size_t bytes = off * 4;
    if (bytes > c->h_map_cap) {
        // the previous plan's kernel may still be retiring (the host returned once its completion
        // word was set): let it finish before its mapped buffer goes
        if (c->h_map) {
            FP_HIP(hipStreamSynchronize(c->stream));
            (void)hipHostFree(c->h_map);
        }
        c->h_map = nullptr;
        c->d_map = nullptr;
        c->h_map_cap = 0;
        const size_t cap = (bytes + bytes / 4 + 4095) & ~(size_t)4095;
        FP_HIP(hipHostMalloc((void **)&c->h_map, cap, hipHostMallocMapped | hipHostMallocCoherent));
        FP_HIP(hipHostGetDevicePointer((void **)&c->d_map, c->h_map, 0));
        c->h_map_cap = cap;
    }
    uint32_t *h = (uint32_t *)c->h_map, *d = (uint32_t *)c->d_map;
    memcpy(h + i_rp, g->row_ptr, (size_t)(V + 1) * 4);
    if (E) memcpy(h + i_col, g->col, (size_t)E * 4);
    memcpy(h + i_hd, g->has_deps, V);
    if (place) {
        memcpy(h + i_cpu, cs->cpu_m, (size_t)V * 4);
        memcpy(h + i_mem, cs->mem_mib, (size_t)V * 4);
        memcpy(h + i_req, cs->req_labels, (size_t)V * 4);
        memcpy(h + i_conf, cs->conflict, (size_t)V * 4);
        if (N) {
            memcpy(h + i_cf, ns->cpu_free, (size_t)N * 4);
            memcpy(h + i_mf, ns->mem_free, (size_t)N * 4);
            memcpy(h + i_lab, ns->labels, (size_t)N * 4);
            memcpy(h + i_cu, ns->conflict_used, (size_t)N * 4);
            memcpy(h + i_sch, ns->schedulable, N);
        }
    }
    h[o_err] = 0xFFFFFFFFu;  // the kernel overwrites it: 0 or -FP_ECORRUPT
    PlanSmallArgs a;
    a.rp = d + i_rp; a.col = d + i_col; a.hd = (const uint8_t *)(d + i_hd);
    a.cpu = d + i_cpu; a.mem = d + i_mem; a.req = d + i_req; a.conf = d + i_conf;
    a.cf = d + i_cf; a.mf = d + i_mf; a.lab = d + i_lab; a.cu = d + i_cu; a.sched = (const uint8_t *)(d + i_sch);
    a.V = V; a.E = E; a.N = N; a.place = place ? 1u : 0u;
    a.perm = d + o_perm; a.level = d + o_lev; a.order = d + o_ord; a.ncyc = d + o_ncyc; a.err = d + o_err;
    a.first = d + o_first; a.count = d + o_count; a.assign = d + o_asg; a.reason = (uint8_t *)(d + o_rsn);
    a.cf_out = d + o_cf; a.mf_out = d + o_mf; a.cu_out = d + o_cu;
    if (lds > 64 * 1024)
        FP_HIP(hipFuncSetAttribute((const void *)k_plan_small, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_LEVEL, &ev);
    k_plan_small<<<1, 1024, lds, c->stream>>>(a);
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_LEVEL, ev);
    // poll the completion word (mapped, coherent host memory); the stream synchronisation is only
    // the fallback for a kernel that has not finished after ~20 ms, and the path when profiling
    volatile uint32_t *done = h + o_err;
    bool seen = false;
    if (!c->profile) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0;; ++spin) {
            if (__atomic_load_n(done, __ATOMIC_ACQUIRE) != 0xFFFFFFFFu) { seen = true; break; }
            if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
        }
    }
    if (!seen) FP_HIP(hipStreamSynchronize(c->stream));
    const uint32_t e = __atomic_load_n(done, __ATOMIC_ACQUIRE);
    if (e == 0xFFFFFFFFu) return FP_EDEVICE;  // the kernel did not finish
    if (e) return -(int)e;
    memcpy(perm_out, h + o_perm, (size_t)V * 4);
    memcpy(level_out, h + o_lev, (size_t)V * 4);
    memcpy(order_out, h + o_ord, (size_t)V * 4);
    if (n_cycle_out) *n_cycle_out = h[o_ncyc];
    if (place) {
        if (first_out) memcpy(first_out, h + o_first, (size_t)V * 4);
        if (count_out) memcpy(count_out, h + o_count, (size_t)V * 4);
        memcpy(assign_out, h + o_asg, (size_t)V * 4);
        memcpy(reason_out, h + o_rsn, V);
        if (N) {
            memcpy(ns->cpu_free, h + o_cf, (size_t)N * 4);
            memcpy(ns->mem_free, h + o_mf, (size_t)N * 4);
            memcpy(ns->conflict_used, h + o_cu, (size_t)N * 4);
        }
    }
    return FP_OK;
}
