// fp_small.h -- the one-workgroup levelizer core (SPEC.md 2.2) shared by k_lvl_small
// (fp_order.hip: fp_levelize / fp_dev_levelize of a small graph) and k_plan_small (fp_small.hip:
// fp_plan_stage, a whole fleet.kdl stage in one launch).
#pragma once
#include "fp_internal.h"

namespace fps {

// a graph of at most LS_V vertices and LS_E edges runs in one workgroup (a round per level costs
// two workgroup barriers, so LS_V bounds the depth too)
constexpr uint32_t LS_V = 512, LS_E = 8192;
// LDS words of ls_levels' scratch: ctl (16), in-degrees, levels and two frontiers (V each), 2 spare
__host__ __device__ inline size_t ls_words(uint32_t V) { return (size_t)V * 4 + 16 + 2; }

// CSR check, in-degrees, level-synchronous Kahn and the stable (level, index) start order of a
// graph of V <= LS_V vertices, by the whole workgroup (every thread calls it; blockDim.x = 1024).
// row_ptr / col / hd may live in global, mapped host or LDS memory; lsm = ls_words(V) words of
// LDS.  Writes level[v] (FP_NONE on / after a cycle) and order[] and returns the number of FP_NONE
// vertices; a corrupt CSR (the general path's k_check_csr / k_indeg conditions) writes nothing and
// returns FP_NONE.  Uniform return; level / order are complete for every thread on return.
__device__ inline uint32_t ls_levels(const uint32_t *row_ptr, const uint32_t *col, const uint8_t *hd, uint32_t V,
                                     uint32_t E, uint32_t *lsm, uint32_t *level, uint32_t *order) {
    // ctl: [0] bad [1] count fr0 [2] count fr1 [3] max level [4] cycle vertices; then deg, lvl and the
    // two frontiers, fr1 with 2 spare words: the key starts reuse fr0 + fr1 (ck + 1 <= V + 2 bins)
    uint32_t *ctl = lsm, *deg = lsm + 16, *lvl = deg + V, *fr0 = lvl + V, *fr1 = fr0 + V;
    const uint32_t t = threadIdx.x, lane = t & 63;
    if (t < 16) ctl[t] = 0u;
    for (uint32_t v = t; v < V; v += blockDim.x) deg[v] = 0u;
    __syncthreads();
    bool bad = false;
    for (uint32_t v = t; v < V; v += blockDim.x) bad |= row_ptr[v + 1] < row_ptr[v];
    if (t == 0) bad |= row_ptr[0] != 0u || row_ptr[V] != E;
    for (uint32_t e = t; e < E; e += blockDim.x) {
        const uint32_t w = col[e];
        if (w >= V) bad = true;
        else atomicAdd(&deg[w], 1u);
    }
    if (bad) atomicOr(&ctl[0], 1u);
    __syncthreads();
    if (ctl[0]) return FP_NONE;  // uniform
    for (uint32_t v = t; v < V; v += blockDim.x) {
        lvl[v] = hd[v] ? 1u : 0u;
        if (deg[v] == 0u) fr0[atomicAdd(&ctl[1], 1u)] = v;
    }
    __syncthreads();
    // level-synchronous Kahn: the frontier in LDS, one round per level
    uint32_t *cur = fr0, *nxt = fr1;
    uint32_t ci = 1;
    while (true) {
        const uint32_t n = ctl[ci];
        if (n == 0u) break;  // uniform (read after the barrier)
        for (uint32_t i = t; i < n; i += blockDim.x) {
            const uint32_t u = cur[i], lu1 = lvl[u] + 1u;
            atomicMax(&ctl[3], lvl[u]);
            for (uint32_t e = row_ptr[u], e1 = row_ptr[u + 1]; e < e1; ++e) {
                const uint32_t w = col[e];
                atomicMax(&lvl[w], lu1);
                if (atomicSub(&deg[w], 1u) == 1u) nxt[atomicAdd(&ctl[3 - ci], 1u)] = w;
            }
        }
        __syncthreads();
        if (t == 0) ctl[ci] = 0u;
        __syncthreads();
        uint32_t *tmp = cur; cur = nxt; nxt = tmp;
        ci = 3 - ci;
    }
    // keys: the level, or the cycle key after every level (max(largest level, 1) + 1)
    const uint32_t maxl = ctl[3];
    const uint32_t ck = (maxl > 1u ? maxl : 1u) + 1u;
    uint32_t *start = fr0;  // both frontiers are free now: 2 V + 2 words for ck + 1 <= V + 2 bins
    for (uint32_t k = t; k <= ck; k += blockDim.x) start[k] = 0u;
    __syncthreads();
    uint32_t nc = 0;
    for (uint32_t v = t; v < V; v += blockDim.x) {
        const bool cy = deg[v] != 0u;
        nc += cy ? 1u : 0u;
        atomicAdd(&start[cy ? ck : lvl[v]], 1u);
    }
    if (nc) atomicAdd(&ctl[4], nc);
    __syncthreads();
    if (t == 0) {  // exclusive scan of <= V + 1 bins (small)
        uint32_t run = 0;
        for (uint32_t k = 0; k <= ck; ++k) { const uint32_t x = start[k]; start[k] = run; run += x; }
    }
    __syncthreads();
    // stable scatter in index order by one wave: equal keys ranked by a ballot match mask
    if (t < 64) {
        const uint32_t nbits = 32u - (uint32_t)__builtin_clz(ck);
        const uint64_t lt = (1ull << lane) - 1ull;
        for (uint32_t v0 = 0; v0 < V; v0 += 64) {
            const uint32_t v = v0 + lane;
            const bool valid = v < V;
            const bool cy = valid && deg[v] != 0u;
            const uint32_t k = valid ? (cy ? ck : lvl[v]) : 0u;
            uint64_t m = __builtin_amdgcn_ballot_w64(valid);
            for (uint32_t b = 0; b < nbits; ++b) {
                const bool bit = (k >> b) & 1u;
                const uint64_t bb = __builtin_amdgcn_ballot_w64(bit);
                m &= bit ? bb : ~bb;
            }
            const uint32_t off = start[k];
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every lane's read before the update
            if (valid) {
                if ((m & lt) == 0) start[k] = off + (uint32_t)__popcll(m);
                order[off + (uint32_t)__popcll(m & lt)] = v;
                level[v] = cy ? FP_NONE : lvl[v];
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
    }
    const uint32_t ncyc = ctl[4];
    __syncthreads();
    return ncyc;
}

}  // namespace fps
