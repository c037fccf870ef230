// fp_place.hip -- stage 3: first-fit-decreasing placement, batched over what-if
// scenarios (SPEC.md 2.3).  One workgroup owns one scenario.
//
// Pipeline per fp_dev_place_batch call:
//   1. k_key_bounds : max(cpu_m), max(mem_mib) over the batch (exact key width)
//   1b. k_value_bitmap + k_rank_tables: when both maxima are below 2^18, the distinct
//                     cpu and mem values of the batch, so that a key field holds the
//                     value's dense rank (order-preserving: the sort is unchanged)
//   2. k_make_keys  : key = (scenario << kb) | ((cmask-c) << mb) | (mmask-m), c/m the
//                     values or their ranks, value = container index; u32 keys when the
//                     fields fit 32 bits, else u64.  Config 4 (512 scenarios, 79 cpu and
//                     256 mem values): 9 + 7 + 8 = 24 bits -> three 8-bit radix passes
//                     instead of five passes over 36-bit u64 keys
//   3. rocprim radix sort (stable) => (cpu desc, mem desc, index asc) per scenario:
//      segmented per scenario when there are several (no scenario bits in the key),
//      device-wide otherwise (or with the scenario field above the key when
//      FLEETPLACE_NO_SEGSORT is set).
//   4. k_ffd_pipe   : (fp_pipe.hip) per scenario, containers in key order stream
//                     through a pipeline of node-group stages (LDS-resident node
//                     tiles); lowest feasible node wins, capacity updated in place.
//   5. k_cost_reduce: packed cost per scenario from the per-segment counters.
#include "fp_internal.h"
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

namespace {

// out[0..1] = max(cpu), max(mem); out[2..3] = min positive cpu, mem (0xFFFFFFFF if none).
// 16-byte loads, a block-level reduction in LDS and one set of atomics per block.
__device__ __forceinline__ void bounds_acc(uint32_t c, uint32_t m, uint32_t &mc, uint32_t &mm, uint32_t &lc,
                                           uint32_t &lm) {
    mc = max(mc, c);
    mm = max(mm, m);
    lc = c ? min(lc, c) : lc;
    lm = m ? min(lm, m) : lm;
}

__global__ __launch_bounds__(256) void k_key_bounds(const uint32_t *__restrict__ cpu,
                                                    const uint32_t *__restrict__ mem, size_t n,
                                                    uint32_t *__restrict__ out /* [4] */) {
    uint32_t mc = 0, mm = 0, lc = 0xFFFFFFFFu, lm = 0xFFFFFFFFu;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool aligned = ((reinterpret_cast<uintptr_t>(cpu) | reinterpret_cast<uintptr_t>(mem)) & 15u) == 0;
    size_t head = 0;
    if (aligned) {
        const size_t n4 = n / 4;
        const uint4 *c4 = reinterpret_cast<const uint4 *>(cpu), *m4 = reinterpret_cast<const uint4 *>(mem);
        for (size_t i = t; i < n4; i += stride) {
            const uint4 c = c4[i], m = m4[i];
            bounds_acc(c.x, m.x, mc, mm, lc, lm);
            bounds_acc(c.y, m.y, mc, mm, lc, lm);
            bounds_acc(c.z, m.z, mc, mm, lc, lm);
            bounds_acc(c.w, m.w, mc, mm, lc, lm);
        }
        head = n4 * 4;
    }
    for (size_t i = head + t; i < n; i += stride) bounds_acc(cpu[i], mem[i], mc, mm, lc, lm);
    for (int o = 32; o > 0; o >>= 1) {
        mc = max(mc, (uint32_t)__shfl_xor((int)mc, o));
        mm = max(mm, (uint32_t)__shfl_xor((int)mm, o));
        lc = min(lc, (uint32_t)__shfl_xor((int)lc, o));
        lm = min(lm, (uint32_t)__shfl_xor((int)lm, o));
    }
    __shared__ uint32_t red[4][4];
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[w][0] = mc; red[w][1] = mm; red[w][2] = lc; red[w][3] = lm; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t q = 1; q < blockDim.x / 64; ++q) {
            mc = max(mc, red[q][0]); mm = max(mm, red[q][1]); lc = min(lc, red[q][2]); lm = min(lm, red[q][3]);
        }
        atomicMax(&out[0], mc);
        atomicMax(&out[1], mm);
        atomicMin(&out[2], lc);
        atomicMin(&out[3], lm);
    }
}

// ---- dense value ranks (order-preserving key compression) ----
constexpr uint32_t RANK_MAX_VALUE = 1u << 18;  // per dimension: 32 KB LDS bitmap
constexpr uint32_t RANK_WORDS = RANK_MAX_VALUE / 32;

// Presence bitmaps of the cpu and mem values (value v -> bit v, v < 2^18), built in LDS
// per block (test before set: after the first few elements almost every bit is already
// there) and ORed into the global bitmaps, nonzero words only.  A value >= 2^18 sets
// *over (the caller then falls back to raw-value keys and k_key_bounds).  The bounds
// the placement needs (max, min positive) come out of the bitmaps (k_rank_tables), so
// this one pass over cpu/mem replaces the bounds pass.
__global__ __launch_bounds__(256) void k_value_bitmap(const uint32_t *__restrict__ cpu,
                                                      const uint32_t *__restrict__ mem, size_t n,
                                                      uint32_t *__restrict__ gbc, uint32_t *__restrict__ gbm,
                                                      uint32_t *__restrict__ over) {
    extern __shared__ uint32_t lbm[];  // [RANK_WORDS] cpu words, then [RANK_WORDS] mem words
    for (uint32_t i = threadIdx.x; i < 2 * RANK_WORDS; i += blockDim.x) lbm[i] = 0;
    __syncthreads();
    uint32_t *lc = lbm, *lm = lbm + RANK_WORDS;
    bool big = false;
    auto add = [&](uint32_t c, uint32_t m) {
        if ((c | m) >= RANK_MAX_VALUE) { big = true; return; }
        const uint32_t bc = 1u << (c & 31), bmk = 1u << (m & 31);
        if (!(lc[c >> 5] & bc)) atomicOr(&lc[c >> 5], bc);
        if (!(lm[m >> 5] & bmk)) atomicOr(&lm[m >> 5], bmk);
    };
    const size_t stride = (size_t)gridDim.x * blockDim.x, t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t head = 0;
    if (((reinterpret_cast<uintptr_t>(cpu) | reinterpret_cast<uintptr_t>(mem)) & 15u) == 0) {
        const uint4 *c4 = reinterpret_cast<const uint4 *>(cpu), *m4 = reinterpret_cast<const uint4 *>(mem);
        for (size_t i = t; i < n / 4; i += stride) {
            const uint4 c = c4[i], m = m4[i];
            add(c.x, m.x); add(c.y, m.y); add(c.z, m.z); add(c.w, m.w);
        }
        head = n / 4 * 4;
    }
    for (size_t i = head + t; i < n; i += stride) add(cpu[i], mem[i]);
    if (__ballot(big) && (threadIdx.x & 63) == 0) atomicOr(over, 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < RANK_WORDS; i += blockDim.x) {
        if (lc[i]) atomicOr(&gbc[i], lc[i]);
        if (lm[i]) atomicOr(&gbm[i], lm[i]);
    }
}

// One block per dimension (blockIdx.x: 0 = cpu, 1 = mem): exclusive prefix popcounts of the
// bitmap words (rank(v) = pre[v >> 5] + popc(bm[v >> 5] & below(v))), the ascending value
// table (val[rank] = v) and the distinct count in cnt[dim].
__global__ __launch_bounds__(1024) void k_rank_tables(const uint32_t *__restrict__ gbc, const uint32_t *__restrict__ gbm,
                                                      uint32_t wc, uint32_t wm, uint32_t *__restrict__ prec,
                                                      uint32_t *__restrict__ prem, uint32_t *__restrict__ valc,
                                                      uint32_t *__restrict__ valm, uint32_t *__restrict__ cnt) {
    const uint32_t *bm = blockIdx.x ? gbm : gbc;
    uint32_t *pre = blockIdx.x ? prem : prec, *val = blockIdx.x ? valm : valc;
    const uint32_t nw = blockIdx.x ? wm : wc;
    const uint32_t per = (nw + blockDim.x - 1) / blockDim.x, w0 = threadIdx.x * per;
    uint32_t local = 0;
    for (uint32_t w = w0; w < w0 + per && w < nw; ++w) local += (uint32_t)__popc(bm[w]);
    __shared__ uint32_t part[1024];
    part[threadIdx.x] = local;
    __syncthreads();
    for (uint32_t o = 1; o < blockDim.x; o <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - local;
    for (uint32_t w = w0; w < w0 + per && w < nw; ++w) {
        pre[w] = run;
        uint32_t x = bm[w];
        while (x) {
            const uint32_t b = (uint32_t)__builtin_ctz(x);
            x &= x - 1;
            val[run++] = w * 32 + b;
        }
    }
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) {
        const uint32_t d = part[threadIdx.x];
        cnt[blockIdx.x] = d;                                       // distinct values
        cnt[2 + blockIdx.x] = d ? val[d - 1] : 0u;                 // max value
        cnt[4 + blockIdx.x] = d == 0 ? 0xFFFFFFFFu : val[0] ? val[0] : d > 1 ? val[1] : 0xFFFFFFFFu;  // min positive
    }
}

__device__ __forceinline__ uint32_t rank_of(uint32_t v, const uint32_t *__restrict__ bm,
                                            const uint32_t *__restrict__ pre) {
    const uint32_t w = v >> 5;
    return pre[w] + (uint32_t)__popc(bm[w] & ((1u << (v & 31)) - 1u));
}

// Key fields are (mask - c) and (mask - m) for descending order, c/m the values (tables
// null) or their dense ranks.
template <class KeyT>
__global__ void k_make_keys(const uint32_t *__restrict__ cpu, const uint32_t *__restrict__ mem,
                            size_t n, uint32_t C, uint32_t kb, uint32_t mb, uint64_t cmax, uint64_t mmax,
                            const uint32_t *__restrict__ bmc, const uint32_t *__restrict__ prec,
                            const uint32_t *__restrict__ bmm, const uint32_t *__restrict__ prem,
                            KeyT *__restrict__ keys, uint32_t *__restrict__ vals) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)i / C, j = (uint32_t)i - s * C;  // n = S * C < 2^32
        const uint64_t sk = kb >= 64 ? 0ull : ((uint64_t)s << kb);
        uint32_t c = cpu[i], m = mem[i];
        if (bmc) {
            c = rank_of(c, bmc, prec);
            m = rank_of(m, bmm, prem);
        }
        keys[i] = (KeyT)(sk | ((cmax - c) << mb) | (mmax - m));
        vals[i] = j;
    }
}

__global__ void k_iota_vals(size_t n, uint32_t C, uint32_t *__restrict__ vals) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        vals[i] = (uint32_t)(i % C);
}

__global__ void k_seg_offsets(uint32_t S, uint32_t C, uint32_t *__restrict__ off) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= S) off[i] = i * C;
}

__global__ void k_fill_cost(uint32_t S, uint32_t scen_base, uint64_t *__restrict__ cost) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < S) cost[s] = fpd::pack_cost(0, 0, scen_base + s);
}

__global__ void k_argmin_cost(const uint64_t *__restrict__ cost, uint32_t n, uint32_t *best) {
    // single block of 1024: min over packed costs; the id field breaks ties
    __shared__ uint64_t red[16];
    uint64_t m = ~0ull;
    uint32_t idx = 0xFFFFFFFFu;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        if (cost[i] < m) { m = cost[i]; idx = i; }
    }
    // pack (cost, idx): costs are unique per scenario id so ties only among equal ids
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t om = __shfl_xor(m, o);
        uint32_t oi = __shfl_xor(idx, o);
        if (om < m || (om == m && oi < idx)) { m = om; idx = oi; }
    }
    __shared__ uint32_t redi[16];
    if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = m; redi[threadIdx.x >> 6] = idx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t bm = ~0ull;
        uint32_t bi = 0xFFFFFFFFu;
        for (uint32_t w = 0; w < (blockDim.x + 63) / 64; ++w)
            if (red[w] < bm || (red[w] == bm && redi[w] < bi)) { bm = red[w]; bi = redi[w]; }
        *best = bi;
    }
}

}  // namespace

// T[0] = 0; T[1..31] spread evenly over the ascending distinct positive values v[0..d)
// (every value is a threshold when there are at most 31)
static void value_thresholds(const uint32_t *v, uint32_t d, uint32_t *T) {
    while (d && v[0] == 0) { ++v; --d; }  // zero is T[0]
    T[0] = 0;
    for (int k = 1; k < FP_BUCKETS; ++k) {
        if (d == 0) { T[k] = 1; continue; }
        const uint64_t i = d <= (uint32_t)(FP_BUCKETS - 1) ? (uint64_t)(k - 1 < (int)d ? k - 1 : d - 1)
                                                             : (uint64_t)(k - 1) * (d - 1) / (FP_BUCKETS - 2);
        T[k] = v[i];
    }
}

static inline unsigned grid_for(size_t n, unsigned block) {
    size_t g = (n + block - 1) / block;
    if (g > 65535u * 4) g = 65535u * 4;
    return (unsigned)(g ? g : 1);
}

// Workspace bytes fp_dev_place_batch takes for S scenarios of C containers x N nodes
// (sort_tmp: the sorts' scratch share of it).
static int place_ws_need(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, size_t *need, size_t *sort_tmp_out) {
    hipStream_t st = c->stream;
    const size_t SC = (size_t)S * C;
    // device-wide sorts are sized for the widest key they may take (u64); the
    // segmented fallback is used only when scenario + key bits exceed 64
    size_t sort_tmp = 0, t = 0;
    FP_HIP(rocprim::radix_sort_pairs(nullptr, t, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                     (uint32_t *)nullptr, SC, 0, 64, st));
    sort_tmp = t;
    FP_HIP(rocprim::radix_sort_pairs(nullptr, t, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                     (uint32_t *)nullptr, SC, 0, 32, st));
    sort_tmp = t > sort_tmp ? t : sort_tmp;
    FP_HIP(rocprim::segmented_radix_sort_pairs(nullptr, t, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                               (uint32_t *)nullptr, (uint32_t *)nullptr, (unsigned)SC, S,
                                               (uint32_t *)nullptr, (uint32_t *)nullptr, 0, 32, st));
    sort_tmp = t > sort_tmp ? t : sort_tmp;
    FP_HIP(rocprim::segmented_radix_sort_pairs(nullptr, t, (uint64_t *)nullptr,
                                               (uint64_t *)nullptr, (uint32_t *)nullptr,
                                               (uint32_t *)nullptr, (unsigned)SC, S,
                                               (uint32_t *)nullptr, (uint32_t *)nullptr, 0, 64, st));
    sort_tmp = t > sort_tmp ? t : sort_tmp;
    const size_t pipe_ws = fp_pipe_ws_bytes(c, S, C, N);
    if (pipe_ws == 0) return FP_EOVERFLOW;
    const size_t rank_ws = 2 * (2 * RANK_WORDS * 4 + RANK_MAX_VALUE * 4) + 2 * 256;
    *need = SC * (8 * 2 + 4 * 2) + (S + 1) * 4 + sort_tmp + pipe_ws + rank_ws + 16 * 256;
    *sort_tmp_out = sort_tmp;
    return FP_OK;
}

int fp_place_ws_bytes_impl(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, uint64_t *bytes) {
    if (S == 0 || C == 0) { *bytes = 0; return FP_OK; }
    if ((size_t)S * C > 0xFFFFFFFFull) return FP_EOVERFLOW;
    size_t need = 0, sort_tmp = 0;
    if (int rc = place_ws_need(c, S, C, N, &need, &sort_tmp)) return rc;
    *bytes = need;
    return FP_OK;
}

int fp_dev_place_batch_impl(fp_ctx *c, const fp_batch *b) {
    const uint32_t S = b->n_scen, C = b->n_containers, N = b->n_nodes;
    if (S == 0) return FP_OK;
    // the packed cost keeps 16 bits of the global scenario id (SPEC.md 2.4): more
    // scenarios would let a wrapped id win a tie it must lose
    if ((uint64_t)b->scen_base + S > 65536ull) return FP_EOVERFLOW;
    hipStream_t st = c->stream;
    if (C == 0) {  // nothing to place: every scenario costs (0 rejected, 0 nodes used)
        if (b->cost) {
            k_fill_cost<<<(S + 255) / 256, 256, 0, st>>>(S, b->scen_base, b->cost);
            FP_HIP(hipGetLastError());
        }
        return FP_OK;
    }
    const size_t SC = (size_t)S * C;
    if (SC > 0xFFFFFFFFull) return FP_EOVERFLOW;  // rocprim segmented sort takes u32 sizes
    if (!b->cpu_m || !b->mem_mib || !b->req_labels || !b->conflict || !b->assign || !b->reason)
        return FP_EINVAL;
    if (N && (!b->cpu_free || !b->mem_free || !b->labels || !b->conflict_used || !b->schedulable))
        return FP_EINVAL;

    // ---- workspace ----
    size_t need = 0, sort_tmp = 0;
    if (int rc0 = place_ws_need(c, S, C, N, &need, &sort_tmp)) return rc0;
    int rc = fp_ws_reserve(c, need);
    if (rc) return rc;
    fp_ws_reset(c);
    uint64_t *keys_in = (uint64_t *)fp_ws_take(c, SC * 8);
    uint64_t *keys_out = (uint64_t *)fp_ws_take(c, SC * 8);
    uint32_t *vals_in = (uint32_t *)fp_ws_take(c, SC * 4);
    uint32_t *vals_out = (uint32_t *)fp_ws_take(c, SC * 4);
    uint32_t *offs = (uint32_t *)fp_ws_take(c, (S + 1) * 4);
    void *tmp = fp_ws_take(c, sort_tmp + 16);
    uint32_t *bounds = (uint32_t *)fp_ws_take(c, 16);
    // rank tables: bitmaps + prefix counts [2][RANK_WORDS] each, value tables, counts
    uint32_t *rbm = (uint32_t *)fp_ws_take(c, 2 * RANK_WORDS * 4);
    uint32_t *rpre = (uint32_t *)fp_ws_take(c, 2 * RANK_WORDS * 4);
    uint32_t *rval = (uint32_t *)fp_ws_take(c, 2 * RANK_MAX_VALUE * 4);
    uint32_t *rcnt = (uint32_t *)fp_ws_take(c, 32);
    if (!keys_in || !keys_out || !vals_in || !vals_out || !offs || !tmp || !bounds || !rbm || !rpre || !rval ||
        !rcnt)
        return FP_ENOMEM;

    // ---- 1-3: FFD order ----
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_SORT, &ev);
    // value bitmaps -> dense ranks, distinct counts and bounds in one pass (values < 2^18)
    FP_HIP(hipMemsetAsync(rbm, 0, 2 * RANK_WORDS * 4, st));
    FP_HIP(hipMemsetAsync(rcnt, 0, 32, st));
    {
        unsigned gb = grid_for((SC + 3) / 4, 256);
        if (gb > 1024) gb = 1024;  // each block merges its bitmaps once
        FP_HIP(hipFuncSetAttribute((const void *)k_value_bitmap, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(2 * RANK_WORDS * 4)));
        k_value_bitmap<<<gb, 256, 2 * RANK_WORDS * 4, st>>>(b->cpu_m, b->mem_mib, SC, rbm, rbm + RANK_WORDS, rcnt + 6);
        FP_HIP(hipGetLastError());
        k_rank_tables<<<2, 1024, 0, st>>>(rbm, rbm + RANK_WORDS, RANK_WORDS, RANK_WORDS, rpre, rpre + RANK_WORDS, rval,
                                          rval + RANK_MAX_VALUE, rcnt);
        FP_HIP(hipGetLastError());
    }
    FP_HIP(hipMemcpyAsync(c->h_small, rcnt, 28, hipMemcpyDeviceToHost, st));
    FP_HIP(hipStreamSynchronize(st));
    const uint32_t *hs = (const uint32_t *)c->h_small;
    const bool ranks = hs[6] == 0;
    uint32_t maxc = hs[2], maxm = hs[3], minc = hs[4], minm = hs[5];
    const uint32_t dc = hs[0], dm = hs[1];
    if (!ranks) {  // a value >= 2^18: raw-value keys, exact bounds
        FP_HIP(hipMemsetAsync(bounds, 0, 8, st));
        FP_HIP(hipMemsetAsync(bounds + 2, 0xFF, 8, st));
        k_key_bounds<<<grid_for((SC + 3) / 4, 256) < 2048 ? grid_for((SC + 3) / 4, 256) : 2048, 256, 0, st>>>(
            b->cpu_m, b->mem_mib, SC, bounds);
        FP_HIP(hipGetLastError());
        FP_HIP(hipMemcpyAsync(c->h_small, bounds, 16, hipMemcpyDeviceToHost, st));
        FP_HIP(hipStreamSynchronize(st));
        maxc = hs[0]; maxm = hs[1]; minc = hs[2]; minm = hs[3];
    }
    uint32_t cbits = fp_bitwidth(maxc), mbits = fp_bitwidth(maxm);
    // dense ranks as key fields (a nonzero key only)
    const uint32_t *bmc = nullptr, *bmm = nullptr, *prc = nullptr, *prm = nullptr;
    const uint32_t *cval = nullptr, *mval = nullptr;
    if (ranks && cbits + mbits > 0) {
        if (dc == 0 || dm == 0) return FP_EDEVICE;  // SC > 0: at least one value each
        bmc = rbm; bmm = rbm + RANK_WORDS; prc = rpre; prm = rpre + RANK_WORDS;
        cval = rval; mval = rval + RANK_MAX_VALUE;
        cbits = fp_bitwidth(dc - 1);
        mbits = fp_bitwidth(dm - 1);
    }
    const uint32_t kbits = cbits + mbits;
    const uint64_t cmax = cbits ? ((cbits == 64 ? ~0ull : ((1ull << cbits) - 1))) : 0ull;
    const uint64_t mmax = mbits ? ((1ull << mbits) - 1) : 0ull;
    const uint32_t sbits = fp_bitwidth(S - 1);
    const uint32_t *order = nullptr;
    const void *skeys = nullptr;
    uint32_t key_bytes = 8;
    if (kbits == 0) {
        k_iota_vals<<<grid_for(SC, 256), 256, 0, st>>>(SC, C, vals_out);
        FP_HIP(hipGetLastError());
        order = vals_out;
    } else if (kbits <= 32 && S > 1 && !getenv("FLEETPLACE_NO_SEGSORT")) {
        // many scenarios: per-scenario segments, so the key holds no scenario field (config 4:
        // 15 bits of radix instead of 27; sort 7.3 -> 5.4 ms for 4096 x 50k)
        uint32_t *k_in = (uint32_t *)keys_in, *k_out = (uint32_t *)keys_out;
        k_make_keys<uint32_t><<<grid_for(SC, 256), 256, 0, st>>>(b->cpu_m, b->mem_mib, SC, C, 64, mbits, cmax, mmax,
                                                                 bmc, prc, bmm, prm, k_in, vals_in);
        FP_HIP(hipGetLastError());
        k_seg_offsets<<<(S + 1 + 255) / 256, 256, 0, st>>>(S, C, offs);
        FP_HIP(hipGetLastError());
        FP_HIP(rocprim::segmented_radix_sort_pairs(tmp, sort_tmp, k_in, k_out, vals_in, vals_out, (unsigned)SC, S,
                                                   offs, offs + 1, 0, kbits, st));
        order = vals_out;
        skeys = k_out;
        key_bytes = 4;
    } else if (kbits + sbits <= 32) {
        uint32_t *k_in = (uint32_t *)keys_in, *k_out = (uint32_t *)keys_out;
        k_make_keys<uint32_t><<<grid_for(SC, 256), 256, 0, st>>>(b->cpu_m, b->mem_mib, SC, C, kbits, mbits, cmax,
                                                                 mmax, bmc, prc, bmm, prm, k_in, vals_in);
        FP_HIP(hipGetLastError());
        FP_HIP(rocprim::radix_sort_pairs(tmp, sort_tmp, k_in, k_out, vals_in, vals_out, SC, 0, kbits + sbits, st));
        order = vals_out;
        skeys = k_out;
        key_bytes = 4;
    } else if (kbits + sbits <= 64) {
        k_make_keys<uint64_t><<<grid_for(SC, 256), 256, 0, st>>>(b->cpu_m, b->mem_mib, SC, C, kbits, mbits, cmax,
                                                                 mmax, bmc, prc, bmm, prm, keys_in, vals_in);
        FP_HIP(hipGetLastError());
        FP_HIP(rocprim::radix_sort_pairs(tmp, sort_tmp, keys_in, keys_out, vals_in, vals_out, SC, 0,
                                         kbits + sbits, st));
        order = vals_out;
        skeys = keys_out;
    } else {
        // full-width cpu and mem (64 key bits): per-scenario segments
        k_make_keys<uint64_t><<<grid_for(SC, 256), 256, 0, st>>>(b->cpu_m, b->mem_mib, SC, C, 64, mbits, cmax,
                                                                 mmax, bmc, prc, bmm, prm, keys_in, vals_in);
        FP_HIP(hipGetLastError());
        k_seg_offsets<<<(S + 1 + 255) / 256, 256, 0, st>>>(S, C, offs);
        FP_HIP(hipGetLastError());
        FP_HIP(rocprim::segmented_radix_sort_pairs(tmp, sort_tmp, keys_in, keys_out, vals_in,
                                                   vals_out, (unsigned)SC, S, offs, offs + 1, 0,
                                                   kbits, st));
        order = vals_out;
        skeys = keys_out;
    }
    fp_prof_end(c, FP_K_SORT, ev);

    // ---- bucket thresholds of the pipeline's candidate masks ----
    // With dense ranks the batch's distinct demand values are known (cval/mval): the
    // thresholds are spread evenly over them, so every bucket spans about D / 31 distinct
    // values (config 4: 79 cpu and 256 mem values -> 2.5 and 8 per bucket).  Geometric
    // steps from min to max spanned 9 and 43 values per bucket at the top of the range,
    // where most demands lie, and the loose buckets cost exact checks that miss.
    // Otherwise (values >= 2^18): geometric from the smallest positive to the largest demand.
    uint32_t tc[FP_BUCKETS], tm[FP_BUCKETS];
    if (cval) {
        std::vector<uint32_t> hv((size_t)dc + dm);
        FP_HIP(hipMemcpyAsync(hv.data(), cval, (size_t)dc * 4, hipMemcpyDeviceToHost, st));
        FP_HIP(hipMemcpyAsync(hv.data() + dc, mval, (size_t)dm * 4, hipMemcpyDeviceToHost, st));
        FP_HIP(hipStreamSynchronize(st));
        value_thresholds(hv.data(), dc, tc);
        value_thresholds(hv.data() + dc, dm, tm);
    } else {
        fp_thresholds(minc == 0xFFFFFFFFu ? 1u : minc, maxc, tc);
        fp_thresholds(minm == 0xFFFFFFFFu ? 1u : minm, maxm, tm);
    }

    // ---- 4-5: placement + cost ----
    return fp_pipe_launch(c, S, C, N, b->scen_base, order, skeys, key_bytes, mbits, cmax, mmax, cval, mval, b, tc, tm);
}

extern "C" int fp_dev_argmin_cost(fp_ctx *c, const uint64_t *cost, uint32_t n, uint32_t *best) {
    if (!c || !cost || !best || n == 0) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    k_argmin_cost<<<1, 1024, 0, c->stream>>>(cost, n, best);
    FP_HIP(hipGetLastError());
    return FP_OK;
}
