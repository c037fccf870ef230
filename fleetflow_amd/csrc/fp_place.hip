// fp_place.hip -- stage 3: first-fit-decreasing placement, batched over what-if
// scenarios (SPEC.md 2.3).  One workgroup owns one scenario.
//
// Pipeline per fp_dev_place_batch call -- asynchronous: every data-dependent choice (dense ranks,
// the LDS sort's eligibility, the key range, the bucket thresholds) is made on the device, so the
// host enqueues the whole call without reading anything back.
//   1. k_value_bitmap + k_rank_tables: the distinct cpu and mem values of a sample (the first
//      THR_SAMPLE scenarios; values below 2^18) as presence bitmaps -> ascending value tables; the
//      raw bounds (max, smallest positive) in the same pass
//   2. k_thresholds: the pipeline's bucket thresholds (spread over the distinct values, or
//      geometric between the bounds), into device memory
//   3a. scenarios of at most ~50k containers (host-known): k_sort_image (the sample's ranks in
//      LDS layout), then the per-scenario LDS sort below (k_scen_sort: digits are ranks in the
//      sample's value set, or in the scenario's own when it holds a value the sample lacks), which
//      falls back, in the same workgroup, to a generic stable LSD sort of the raw values when the
//      scenario has more than 256 distinct values or values >= 2^18
//   3b. larger scenarios: k_make_keys (full-width key (~cpu << 32 | ~mem), value = index) and a
//      stable rocprim radix sort over 64 bits, segmented per scenario when there are several
//   4. k_ffd_pipe   : (fp_pipe.hip) per scenario, containers in key order stream
//                     through a pipeline of node-group stages (LDS-resident node
//                     tiles); lowest feasible node wins, capacity updated in place.
//   5. k_cost_reduce: packed cost per scenario from the per-segment counters.
#include "fp_internal.h"
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

namespace {

// running max and smallest positive value of cpu (mc, lc) and mem (mm, lm)
__device__ __forceinline__ void bounds_acc(uint32_t c, uint32_t m, uint32_t &mc, uint32_t &mm, uint32_t &lc,
                                           uint32_t &lm) {
    mc = max(mc, c);
    mm = max(mm, m);
    lc = c ? min(lc, c) : lc;
    lm = m ? min(lm, m) : lm;
}


// ---- dense value ranks (order-preserving key compression) ----
constexpr uint32_t RANK_MAX_VALUE = 1u << 18;  // per dimension: 32 KB LDS bitmap
constexpr uint32_t RANK_WORDS = RANK_MAX_VALUE / 32;

// Presence bitmaps of the cpu and mem values (value v -> bit v, v < 2^18), built in LDS
// per block (test before set: after the first few elements almost every bit is already
// there) and ORed into the global bitmaps, nonzero words only.  A value >= 2^18 sets
// cnt[CN_OVER] (the thresholds are then geometric).  The raw bounds come out of the same pass: cnt[CN_MAXC..CN_MINM]
// (max cpu, max mem, smallest positive cpu, mem; the minima start at 0xFFFFFFFF).
// CN_ORC / CN_ORM: the OR of every cpu / mem value of the batch (containers here, schedulable nodes in
// k_node_summary): the packed-capacity decision of k_ffd_pipe (fp_pipe_pk.h)
enum { CN_DC = 0, CN_DM = 1, CN_OVER = 6, CN_MAXC = 8, CN_MAXM = 9, CN_MINC = 10, CN_MINM = 11, CN_ORC = 12, CN_ORM = 13,
       CN_WORDS = 16 };
__global__ __launch_bounds__(256) void k_value_bitmap(const uint32_t *__restrict__ cpu,
                                                      const uint32_t *__restrict__ mem, size_t n,
                                                      uint32_t *__restrict__ gbc, uint32_t *__restrict__ gbm,
                                                      uint32_t *__restrict__ cnt) {
    extern __shared__ uint32_t lbm[];  // [RANK_WORDS] cpu words, then [RANK_WORDS] mem words
    for (uint32_t i = threadIdx.x; i < 2 * RANK_WORDS; i += blockDim.x) lbm[i] = 0;
    __syncthreads();
    uint32_t *lc = lbm, *lm = lbm + RANK_WORDS;
    bool big = false;
    uint32_t bxc = 0, bxm = 0, bnc = 0xFFFFFFFFu, bnm = 0xFFFFFFFFu;
    auto add = [&](uint32_t c, uint32_t m) {
        bounds_acc(c, m, bxc, bxm, bnc, bnm);
        if ((c | m) >= RANK_MAX_VALUE) { big = true; return; }
        const uint32_t bc = 1u << (c & 31), bmk = 1u << (m & 31);
        if (!(lc[c >> 5] & bc)) atomicOr(&lc[c >> 5], bc);
        if (!(lm[m >> 5] & bmk)) atomicOr(&lm[m >> 5], bmk);
    };
    const size_t stride = (size_t)gridDim.x * blockDim.x, t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t head = 0;
    if (((reinterpret_cast<uintptr_t>(cpu) | reinterpret_cast<uintptr_t>(mem)) & 15u) == 0) {
        const uint4 *c4 = reinterpret_cast<const uint4 *>(cpu), *m4 = reinterpret_cast<const uint4 *>(mem);
        const size_t n4 = n / 4;
        // BM_UNROLL 16-B loads of each array in flight per thread: the 64 KB of LDS bitmaps allow
        // two blocks per CU, too few waves to cover HBM latency one load pair at a time
        constexpr uint32_t BM_UNROLL = 4;
        for (size_t i0 = t; i0 < n4; i0 += BM_UNROLL * stride) {
            uint4 c[BM_UNROLL], m[BM_UNROLL];
#pragma unroll
            for (uint32_t u = 0; u < BM_UNROLL; ++u) {
                const size_t i = i0 + u * stride;
                if (i < n4) { c[u] = c4[i]; m[u] = m4[i]; }
            }
#pragma unroll
            for (uint32_t u = 0; u < BM_UNROLL; ++u) {
                if (i0 + u * stride < n4) { add(c[u].x, m[u].x); add(c[u].y, m[u].y); add(c[u].z, m[u].z); add(c[u].w, m[u].w); }
            }
        }
        head = n4 * 4;
    }
    for (size_t i = head + t; i < n; i += stride) add(cpu[i], mem[i]);
    // block reductions, then at most one atomic per block and word, and none that would change
    // nothing: per-wave atomics on these few words serialise at the memory side
    const bool anybig = __syncthreads_or(big);
    for (int o = 32; o > 0; o >>= 1) {
        bxc = max(bxc, (uint32_t)__shfl_xor((int)bxc, o));
        bxm = max(bxm, (uint32_t)__shfl_xor((int)bxm, o));
        bnc = min(bnc, (uint32_t)__shfl_xor((int)bnc, o));
        bnm = min(bnm, (uint32_t)__shfl_xor((int)bnm, o));
    }
    __shared__ uint32_t wb[4][4];  // [wave][max c, max m, min c, min m], 256 threads
    if ((threadIdx.x & 63) == 0) {
        wb[threadIdx.x >> 6][0] = bxc; wb[threadIdx.x >> 6][1] = bxm;
        wb[threadIdx.x >> 6][2] = bnc; wb[threadIdx.x >> 6][3] = bnm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 1; w < 4; ++w) {
            bxc = max(bxc, wb[w][0]); bxm = max(bxm, wb[w][1]);
            bnc = min(bnc, wb[w][2]); bnm = min(bnm, wb[w][3]);
        }
        auto ld = [](uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        if (anybig && !ld(&cnt[CN_OVER])) atomicOr(&cnt[CN_OVER], 1u);
        if (bxc > ld(&cnt[CN_MAXC])) atomicMax(&cnt[CN_MAXC], bxc);
        if (bxm > ld(&cnt[CN_MAXM])) atomicMax(&cnt[CN_MAXM], bxm);
        if (bnc < ld(&cnt[CN_MINC])) atomicMin(&cnt[CN_MINC], bnc);
        if (bnm < ld(&cnt[CN_MINM])) atomicMin(&cnt[CN_MINM], bnm);
    }
    for (uint32_t i = threadIdx.x; i < RANK_WORDS; i += blockDim.x) {
        if (lc[i] & ~gbc[i]) atomicOr(&gbc[i], lc[i]);
        if (lm[i] & ~gbm[i]) atomicOr(&gbm[i], lm[i]);
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

// Radix-path keys: (~cpu << 32) | ~mem (descending demands sort ascending), value = the index in
// the scenario.
// Also ORs every value into rng[0] (cpu) / rng[1] (mem): one atomic per block and word.
__global__ __launch_bounds__(256) void k_make_keys(const uint32_t *__restrict__ cpu, const uint32_t *__restrict__ mem,
                                                   size_t n, uint32_t C, uint64_t *__restrict__ keys,
                                                   uint32_t *__restrict__ vals, uint32_t *__restrict__ rng) {
    uint32_t oc = 0, om = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)i / C, j = (uint32_t)i - s * C;  // n = S * C < 2^32
        const uint32_t c = cpu[i], m = mem[i];
        keys[i] = ((uint64_t)~c << 32) | (uint32_t)~m;
        vals[i] = j;
        oc |= c;
        om |= m;
    }
    for (int o = 32; o > 0; o >>= 1) {
        oc |= (uint32_t)__shfl_xor((int)oc, o);
        om |= (uint32_t)__shfl_xor((int)om, o);
    }
    __shared__ uint32_t red[2];
    if (threadIdx.x < 2) red[threadIdx.x] = 0u;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        atomicOr(&red[0], oc);
        atomicOr(&red[1], om);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        fp_or_new_bits(&rng[0], red[0]);
        fp_or_new_bits(&rng[1], red[1]);
    }
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

// ---- per-scenario LDS sort (scenarios of at most ~50k containers) ----
//
// Every scenario is sorted into FFD order (cpu desc, mem desc, index asc) by one workgroup
// of 1024 threads in LDS.  It writes the order and the sorted cpu / mem / position words
// itself, so no radix keys, onesweep passes or key decode touch HBM.  The digits are value ranks
// in a set that holds every value of the scenario, flipped so that an ascending digit means a
// descending demand: hd = dc-1-rank(cpu), ld = dm-1-rank(mem), each below 256.  k_scen_sort, one
// workgroup per scenario:
//   R   presence bitmaps of the value set (v < 2^18) in LDS, their prefix popcounts and the value
//       of every rank.  Pass 0 copies the sample's (k_sort_image); a value of the scenario outside
//       it (found in A0) sends the workgroup to pass 1, the scenario's own values from one
//       streaming pass: dc, dm and the eligibility of the digit sort (<= 256 values per
//       dimension) are then the scenario's own, decided in the workgroup
//   A0  each wave loads its contiguous slice of the scenario, ranks it into digit pairs (kept in
//       registers), keeps ld[j] in LDS and counts the hd digits (packed u16 LDS atomics); one
//       scan gives every (wave, digit) its offset
//   A1  each wave walks its slice in order, 64 containers at a time; a container's place
//       among equal digits in the 64 is a match mask of ballots, so X[p] = index in
//       stable hd order with no barrier inside the pass
//   B   every hd bucket (~630 containers in config 4) is sorted by ld by one wave, stable
//       the same way, and written straight to its final positions; the bucket's window of
//       each output array is a few KB, so its scattered dword stores merge in L2
// A scenario without such digits takes the generic fallback (ss_generic) in the same workgroup.
// Round 3 ranked against the whole batch's values instead: two streaming passes over every
// container (k_value_bitmap, k_digits: 0.85 ms per 4096-scenario step) before the sort.
// LDS: max(X u16[C], the rank tables' 96 KB) + ld u8[C] + [16][256] u16 + tables -> C <= 50,336.
constexpr uint32_t SS_DIG = 256;     // digits per dimension (dense ranks)
constexpr uint32_t SS_WAVES = 16;
constexpr uint32_t SS_CHUNKS = 50;   // 64-container chunks per wave slice: C <= 16 x 50 x 64 = 51,200
constexpr uint32_t SS_LB = 25;       // chunks whose loads are in flight together (R, A0)
constexpr uint32_t SS_REG = 16;      // B: buckets of up to 64 x SS_REG containers are reordered in registers
constexpr size_t SS_LDS_CAP = 160 * 1024;
constexpr uint32_t SR_W = RANK_WORDS;                  // bitmap words per dimension (values < 2^18)
constexpr size_t SR_BYTES = (size_t)SR_W * (4 + 2) * 2;  // bitmaps u32 + prefix counts u16, both dimensions
constexpr size_t SS_TAB_BYTES = SS_DIG * (4 + 4 + 1 + 1);  // MV, CV u32 and MB, CB u8 per digit
constexpr size_t SS_IMG_BYTES = SR_BYTES + SS_TAB_BYTES;

__host__ __device__ static inline size_t ss_align16(size_t b) { return (b + 15) & ~(size_t)15; }
__host__ __device__ static inline size_t ss_xr_bytes(uint32_t C) {
    return ss_align16((size_t)C * 2 > SR_BYTES ? (size_t)C * 2 : SR_BYTES);
}
// XR (X / rank tables), LD, WH [16][256] u16, HS/HB u32 [256], MV/CV u32 [256], MB/CB u8 [256], NEXT [4]
static inline size_t ss_lds_bytes(uint32_t C) {
    return ss_xr_bytes(C) + ss_align16(C) + SS_WAVES * SS_DIG * 2 + 2 * SS_DIG * 4 + 2 * SS_DIG * 4 + 2 * SS_DIG + 16;
}

struct ScenSortArgs {
    uint32_t C, kpack;
    const uint32_t *cpu, *mem;               // [S][C] the demands
    uint32_t *order, *s_cpu, *s_mem, *s_idx; // [S][C] FFD order, sorted cpu / mem / position word
    const uint32_t *T;                       // [2 FP_BUCKETS] bucket thresholds (cpu, then mem; device)
    const uint32_t *scnt;                    // the sample's counts (CN_*)
    const unsigned char *simg;               // the sample's LDS image (k_sort_image), SS_IMG_BYTES
    uint32_t *rng;                           // [2] the batch's OR of every cpu / mem value (CN_ORC)
};

// the u16 digit rows are also counted, zeroed and scanned through 32/64-bit views: these
// types may alias the u16 entries (else type-based alias analysis may reorder them)
typedef uint64_t __attribute__((may_alias)) ss_u64a;
typedef uint32_t __attribute__((may_alias)) ss_u32a;
typedef uint32_t ss_u32x4 __attribute__((ext_vector_type(4)));

// lanes holding the same digit as this lane (among `valid` lanes); digits < 2^nb
__device__ __forceinline__ uint64_t ss_match(uint32_t v, bool valid, uint32_t nb) {
    uint64_t m = __builtin_amdgcn_ballot_w64(valid);
    for (uint32_t b = 0; b < nb; ++b) {
        const bool bit = (v >> b) & 1u;
        const uint64_t bb = __builtin_amdgcn_ballot_w64(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

__device__ __forceinline__ uint32_t ss_bucket(const uint32_t *t, uint32_t v) {
    uint32_t k = 0;
#pragma unroll
    for (uint32_t step = FP_BUCKETS / 2; step; step >>= 1) k += t[k + step] <= v ? step : 0u;
    return k;
}

// +1 on the u16 counter `d` of a packed row (two counters per dword; counts stay < 2^16)
__device__ __forceinline__ void ss_inc16(uint16_t *row, uint32_t d) {
    atomicAdd(reinterpret_cast<ss_u32a *>(row) + (d >> 1), 1u << ((d & 1u) * 16u));
}

// exclusive scan of a 256-entry u16 row (4 entries per lane) from `base`, in place
__device__ __forceinline__ void ss_row_scan(uint16_t *row, uint32_t lane, uint32_t base) {
    const uint64_t q = reinterpret_cast<ss_u64a *>(row)[lane];
    const uint32_t c0 = (uint32_t)(q & 0xFFFF), c1 = (uint32_t)((q >> 16) & 0xFFFF), c2 = (uint32_t)((q >> 32) & 0xFFFF);
    const uint32_t sum = c0 + c1 + c2 + (uint32_t)(q >> 48);
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        inc += lane >= (uint32_t)o ? y : 0u;
    }
    const uint64_t e0 = base + inc - sum;
    reinterpret_cast<ss_u64a *>(row)[lane] = e0 | ((e0 + c0) << 16) | ((e0 + c0 + c1) << 32) | ((e0 + c0 + c1 + c2) << 48);
}

// exclusive (wave, digit) offsets of a pass in wave order from the per-wave counts in WH: bucket
// starts in HS, ends in HB (the scheme of k_scen_sort's A0 -> A1)
__device__ __forceinline__ void ss_offsets(uint16_t *WH, uint32_t *HS, uint32_t *HB, uint32_t t, uint32_t lane,
                                           uint32_t w) {
    if (t < SS_DIG) {  // totals per digit (thread t = digit t)
        uint32_t s = 0;
#pragma unroll
        for (uint32_t ww = 0; ww < SS_WAVES; ++ww) s += WH[ww * SS_DIG + t];
        HB[t] = s;
    }
    __syncthreads();
    if (w == 0) {  // bucket starts: exclusive scan of the totals (4 per lane)
        const uint32_t c0 = HB[4 * lane], c1 = HB[4 * lane + 1], c2 = HB[4 * lane + 2], c3 = HB[4 * lane + 3];
        const uint32_t sum = c0 + c1 + c2 + c3;
        uint32_t inc = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
            inc += lane >= (uint32_t)o ? y : 0u;
        }
        const uint32_t ex = inc - sum;
        HS[4 * lane] = ex;
        HS[4 * lane + 1] = ex + c0;
        HS[4 * lane + 2] = ex + c0 + c1;
        HS[4 * lane + 3] = ex + c0 + c1 + c2;
    }
    __syncthreads();
    if (t < SS_DIG) {  // (wave, digit) offsets in wave order; HB = bucket ends
        uint32_t run = HS[t];
#pragma unroll
        for (uint32_t ww = 0; ww < SS_WAVES; ++ww) {
            const uint32_t c = WH[ww * SS_DIG + t];
            WH[ww * SS_DIG + t] = (uint16_t)run;
            run += c;
        }
        HB[t] = run;
    }
    __syncthreads();
}

// The generic fallback of k_scen_sort (a batch without dense ranks: more than 256 distinct cpu or
// mem values, or a value >= 2^18): the same (cpu desc, mem desc, index asc) order by a stable LSD
// sort over the bytes of ~mem, then of ~cpu (ascending ~v = descending v), eight counting passes
// with A0 / A1's per-wave scheme.  Pass k writes the order to X (LDS) when k is even and to this
// scenario's `order` row when k is odd (pass 0 starts from the identity), so pass 7 leaves it in
// `order`; a pass reads the row back through agent-scope loads (other waves of the workgroup wrote
// it in the pass before).  Then the sorted fields as the fast path writes them.
__device__ void ss_generic(const ScenSortArgs &a, uint16_t *X, uint16_t *WH, uint32_t *HS, uint32_t *HB,
                           size_t cb, uint32_t C) {
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t L = (C + SS_WAVES - 1) / SS_WAVES;
    const uint32_t s0 = min(C, w * L), s1 = min(C, s0 + L);
    uint16_t *myrow = WH + w * SS_DIG;
    uint32_t *ord = a.order + cb;
    const uint32_t *cpu = a.cpu + cb, *mem = a.mem + cb;
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t *key = k < 4 ? mem : cpu;
        const uint32_t sh = 8u * (k & 3u);
        auto src = [&](uint32_t p) -> uint32_t {
            return k == 0 ? p
                   : (k & 1u) ? (uint32_t)X[p]
                              : __hip_atomic_load(&ord[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        for (uint32_t i = t; i < SS_WAVES * SS_DIG / 2; i += blockDim.x) reinterpret_cast<ss_u32a *>(WH)[i] = 0u;
        __syncthreads();
        for (uint32_t p = s0 + lane; p < s1; p += 64) ss_inc16(myrow, ((~key[src(p)]) >> sh) & 0xFFu);
        __syncthreads();
        ss_offsets(WH, HS, HB, t, lane, w);
        for (uint32_t p0 = s0; p0 < s1; p0 += 64) {
            const uint32_t p = p0 + lane;
            const bool valid = p < s1;
            const uint32_t j = valid ? src(p) : 0u;
            const uint32_t d = valid ? ((~key[j]) >> sh) & 0xFFu : 0u;
            const uint64_t m = ss_match(d, valid, 8);
            const uint32_t off = myrow[d];
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every lane's read before the update
            if (valid) {
                if ((m & lt) == 0) myrow[d] = (uint16_t)(off + __popcll(m));
                const uint32_t q = off + (uint32_t)__popcll(m & lt);
                if (k & 1u) ord[q] = j;
                else X[q] = (uint16_t)j;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        __syncthreads();
    }
    uint32_t oc = 0, om = 0;  // the batch's OR words (k_scen_sort)
    for (uint32_t P = t; P < C; P += blockDim.x) {
        const uint32_t j = __hip_atomic_load(&ord[P], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t cv = cpu[j], mv = mem[j];
        a.s_cpu[cb + P] = cv;
        a.s_mem[cb + P] = mv;
        a.s_idx[cb + P] = P | (a.kpack ? (ss_bucket(a.T, cv) << 21) | (ss_bucket(a.T + FP_BUCKETS, mv) << 26) : 0u);
        oc |= cv;
        om |= mv;
    }
    for (int o = 32; o > 0; o >>= 1) {
        oc |= (uint32_t)__shfl_xor((int)oc, o);
        om |= (uint32_t)__shfl_xor((int)om, o);
    }
    __syncthreads();  // HS is free: every wave is past the last pass
    if (t < 2) HS[t] = 0u;
    __syncthreads();
    if (lane == 0) {
        atomicOr(&HS[0], oc);
        atomicOr(&HS[1], om);
    }
    __syncthreads();
    if (t == 0) {
        fp_or_new_bits(&a.rng[0], HS[0]);
        fp_or_new_bits(&a.rng[1], HS[1]);
    }
}

#ifdef FP_PIPE_STATS
// diagnostics build: k_scen_sort phase cycles summed over workgroups (fp_debug_sort_stats):
// [0] R (ranks) [1] A0 + offsets [2] A1 [3] B (until the last wave) [4] B busy summed over waves
// [5] workgroups [6] largest bucket [7] whole kernel
__device__ unsigned long long g_sort_stats[8];
#define SS_CLK() __builtin_amdgcn_s_memtime()
#else
#define SS_CLK() 0ull
#endif

// exclusive block scan of one u32 per thread (1024 threads); `part` holds 16 entries
__device__ __forceinline__ uint32_t ss_block_excl(uint32_t v, uint32_t *part, uint32_t lane, uint32_t w,
                                                  uint32_t &total) {
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        inc += lane >= (uint32_t)o ? y : 0u;
    }
    if (lane == 63) part[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (uint32_t ww = 0; ww < SS_WAVES; ++ww) {
        const uint32_t x = part[ww];
        before += ww < w ? x : 0u;
        total += x;
    }
    return before + inc - v;
}

__global__ __launch_bounds__(1024) void k_scen_sort(const ScenSortArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char ssm[];
    const uint32_t C = a.C;
    uint16_t *X = reinterpret_cast<uint16_t *>(ssm);
    uint8_t *LD = ssm + ss_xr_bytes(C);
    uint16_t *WH = reinterpret_cast<uint16_t *>(LD + ss_align16(C));     // [wave][digit]
    uint32_t *HS = reinterpret_cast<uint32_t *>(WH + SS_WAVES * SS_DIG);  // bucket starts
    uint32_t *HB = HS + SS_DIG;                                          // bucket ends
    uint32_t *MV = HB + SS_DIG;                                          // mem value per ld
    uint32_t *CV = MV + SS_DIG;                                          // cpu value per hd
    uint8_t *MB = reinterpret_cast<uint8_t *>(CV + SS_DIG);              // mem bucket per ld
    uint8_t *CB = MB + SS_DIG;                                           // cpu bucket per hd
    uint32_t *NEXT = reinterpret_cast<uint32_t *>(CB + SS_DIG);          // [0] next bucket [1] a value >= 2^18
    // R's tables live where X will be (X is first written in A1)
    uint32_t *BMC = reinterpret_cast<uint32_t *>(ssm), *BMM = BMC + SR_W;
    uint16_t *PRC = reinterpret_cast<uint16_t *>(BMM + SR_W), *PRM = PRC + SR_W;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const size_t cb = (size_t)blockIdx.x * C;
    const uint32_t *cpu = a.cpu + cb, *mem = a.mem + cb;
    const unsigned long long ck0 = SS_CLK();

    // ---- R: the value set the digits rank against.  Pass 0 takes the sample's (k_value_bitmap
    // over the first THR_SAMPLE scenarios: a 64-KB copy from L2) when it has <= 256 values per
    // dimension; A0 then checks that every value of the scenario is in it, and a miss anywhere
    // sends the workgroup to pass 1, the scenario's own distinct values (one streaming pass).  The
    // digits are ranks in either set, so the order is exact either way. ----
    const uint32_t scd = a.scnt[CN_DC], scm = a.scnt[CN_DM];
    const bool samp = a.scnt[CN_OVER] == 0u && scd - 1u < SS_DIG && scm - 1u < SS_DIG;  // grid-uniform
    const uint32_t L = (C + SS_WAVES - 1) / SS_WAVES;
    const uint32_t s0 = min(C, w * L), s1 = min(C, s0 + L);
    uint16_t *myrow = WH + w * SS_DIG;
    uint32_t dc = 0, dm = 0, hbits = 0, lbits = 0;
    uint32_t dvp[SS_CHUNKS / 2];
    unsigned long long ck1 = 0;
    // the scenario's rows as buffer resources: range-checked loads (0 past C) without branches
    const __amdgpu_buffer_rsrc_t rc_cpu = __builtin_amdgcn_make_buffer_rsrc((void *)cpu, (short)0, (int)(4 * C), 0x00020000);
    const __amdgpu_buffer_rsrc_t rc_mem = __builtin_amdgcn_make_buffer_rsrc((void *)mem, (short)0, (int)(4 * C), 0x00020000);
    // the sample's image: 16-B units of BMC, BMM, PRC, PRM up to the largest sample value's word,
    // then the tables; unit u -> image byte offset (returned) and LDS byte offset (dst)
    const uint32_t smc = a.scnt[2], smm = a.scnt[3];  // the sample's largest values (k_rank_tables)
    const uint32_t iwc = (smc >> 5) + 1u, iwm = (smm >> 5) + 1u;
    const uint32_t ib1 = (4u * iwc + 15u) / 16u, ib2 = ib1 + (4u * iwm + 15u) / 16u;
    const uint32_t ib3 = ib2 + (2u * iwc + 15u) / 16u, ib4 = ib3 + (2u * iwm + 15u) / 16u;
    const uint32_t img_units = ib4 + (uint32_t)(SS_TAB_BYTES / 16);
    const uint32_t tab_dst = (uint32_t)(reinterpret_cast<unsigned char *>(MV) - ssm);
    auto img_unit = [&](uint32_t u, uint32_t &dst) -> uint32_t {
        const uint32_t src = u < ib1   ? 16u * u
                             : u < ib2 ? 4u * SR_W + 16u * (u - ib1)
                             : u < ib3 ? 8u * SR_W + 16u * (u - ib2)
                             : u < ib4 ? 10u * SR_W + 16u * (u - ib3)
                                       : (uint32_t)SR_BYTES + 16u * (u - ib4);
        dst = u < ib4 ? src : tab_dst + 16u * (u - ib4);
        return src;
    };
    // one pass (inlined twice): 0 = ranked, 1 = a miss (pass 0 only), 2 = the generic sort ran
    auto rank_pass = [&](const uint32_t pass) -> uint32_t {
        // pass 0: the part of the sample's image the sample's values use (bitmap and prefix words
        // up to the largest value, in LDS layout where X will be; then the value and bucket
        // tables: MV, CV, MB, CB are contiguous and 16-B aligned) is loaded first, one 16-B unit
        // per thread, then A0's first loads are issued, in flight while the image is written
        ss_u32x4 imv;
        uint32_t isrc = 0, idst = 0;
        uint32_t pcv[SS_LB], pmv[SS_LB];
        if (pass == 0) {
            isrc = img_unit(min(t, img_units - 1u), idst);
            imv = *reinterpret_cast<const ss_u32x4 *>(a.simg + isrc);  // no branch (vmcnt)
            __builtin_amdgcn_sched_barrier(0);  // the image's loads stay ahead of A0's (in-order vmcnt)
#pragma unroll
            for (uint32_t k = 0; k < SS_LB; ++k) {  // no branches: the loads stay countable (vmcnt)
                pcv[k] = __builtin_amdgcn_raw_buffer_load_b32(rc_cpu, (int)(4 * (s0 + lane)), (int)(256 * k), 0);
                pmv[k] = __builtin_amdgcn_raw_buffer_load_b32(rc_mem, (int)(4 * (s0 + lane)), (int)(256 * k), 0);
            }
        }
        for (uint32_t i = t; i < SS_WAVES * SS_DIG / 2; i += blockDim.x) reinterpret_cast<ss_u32a *>(WH)[i] = 0u;
        if (t < 4) NEXT[t] = 0u;
        if (pass == 0) {
            if (t < img_units) *reinterpret_cast<ss_u32x4 *>(ssm + idst) = imv;
            for (uint32_t u = t + 1024; u < img_units; u += 1024) {  // sample values above ~2^16
                const uint32_t so = img_unit(u, idst);
                *reinterpret_cast<ss_u32x4 *>(ssm + idst) = *reinterpret_cast<const ss_u32x4 *>(a.simg + so);
            }
            dc = scd;
            dm = scm;
            __syncthreads();
        } else {
            for (uint32_t i = t; i < 2 * SR_W; i += blockDim.x) BMC[i] = 0u;
            __syncthreads();
            bool big = false;
            for (uint32_t k0 = 0; k0 < SS_CHUNKS; k0 += SS_LB) {  // coalesced, SS_LB x 2 loads in flight
                uint32_t cv[SS_LB], mv[SS_LB];
#pragma unroll
                for (uint32_t k = 0; k < SS_LB; ++k) {
                    const uint32_t i = t + blockDim.x * (k0 + k);
                    cv[k] = i < C ? __builtin_nontemporal_load(&cpu[i]) : 0u;
                    mv[k] = i < C ? __builtin_nontemporal_load(&mem[i]) : 0u;
                }
#pragma unroll
                for (uint32_t k = 0; k < SS_LB; ++k) {
                    if (t + blockDim.x * (k0 + k) < C) {
                        const uint32_t c = cv[k], m = mv[k];
                        if ((c | m) >= RANK_MAX_VALUE) {
                            big = true;
                        } else {  // test before set: most bits are already there
                            const uint32_t bc = 1u << (c & 31), bm = 1u << (m & 31);
                            if (!(BMC[c >> 5] & bc)) atomicOr(&BMC[c >> 5], bc);
                            if (!(BMM[m >> 5] & bm)) atomicOr(&BMM[m >> 5], bm);
                        }
                    }
                }
            }
            if (__ballot(big) && lane == 0) atomicOr(&NEXT[1], 1u);
            __syncthreads();
            // prefix popcounts: thread t owns words [8t, 8t + 8) of both bitmaps (SR_W = 8 x 1024)
            static_assert(SR_W == 8 * 1024, "rank words per thread");
            uint32_t bw[8], bx[8], sc = 0, sm = 0;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                bw[j] = BMC[8 * t + j];
                bx[j] = BMM[8 * t + j];
                sc += (uint32_t)__popc(bw[j]);
                sm += (uint32_t)__popc(bx[j]);
            }
            uint32_t pc = ss_block_excl(sc, HS, lane, w, dc);
            __syncthreads();  // HS reused by the second scan
            uint32_t pm = ss_block_excl(sm, HB, lane, w, dm);
            const bool elig = NEXT[1] == 0u && dc >= 1u && dm >= 1u && dc <= SS_DIG && dm <= SS_DIG;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                PRC[8 * t + j] = (uint16_t)pc;
                PRM[8 * t + j] = (uint16_t)pm;
                if (elig) {  // the value of every rank, flipped to digit order (<= 256 bits in all)
                    for (uint32_t x = bw[j]; x; x &= x - 1) CV[dc - 1u - pc++] = (8 * t + j) * 32 + (uint32_t)__builtin_ctz(x);
                    for (uint32_t x = bx[j]; x; x &= x - 1) MV[dm - 1u - pm++] = (8 * t + j) * 32 + (uint32_t)__builtin_ctz(x);
                } else {
                    pc += (uint32_t)__popc(bw[j]);
                    pm += (uint32_t)__popc(bx[j]);
                }
            }
            __syncthreads();
            if (!elig) {  // more than 256 distinct values in a dimension, or a value >= 2^18 (uniform)
                ss_generic(a, X, WH, HS, HB, cb, C);
                return 2u;
            }
            if (t < SS_DIG) {
                MB[t] = a.kpack && t < dm ? (uint8_t)ss_bucket(a.T + FP_BUCKETS, MV[t]) : 0;
                CB[t] = a.kpack && t < dc ? (uint8_t)ss_bucket(a.T, CV[t]) : 0;
            }
        }
        ck1 = SS_CLK();
        // bits of the largest digit (dc - 1, dm - 1): the match masks test only those
        hbits = dc > 1 ? 32u - (uint32_t)__builtin_clz(dc - 1u) : 0u;
        lbits = dm > 1 ? 32u - (uint32_t)__builtin_clz(dm - 1u) : 0u;

        // ---- A0: the wave's slice [s0, s1) ranked into digit pairs (kept in registers, two per
        // dword), ld into LDS, per-wave hd counts; a value outside the set (pass 0) is a miss ----
        bool miss = false;
#pragma unroll
        for (uint32_t k = 0; k < SS_CHUNKS / 2; ++k) dvp[k] = 0u;
#pragma unroll
        for (uint32_t k0 = 0; k0 < SS_CHUNKS; k0 += SS_LB) {
            uint32_t cv[SS_LB], mv[SS_LB];
#pragma unroll
            for (uint32_t k = 0; k < SS_LB; ++k) {
                const uint32_t p = s0 + 64 * (k0 + k) + lane;
                if (pass == 0 && k0 == 0) {
                    cv[k] = pcv[k];
                    mv[k] = pmv[k];
                } else {
                    cv[k] = p < s1 ? __builtin_nontemporal_load(&cpu[p]) : 0u;
                    mv[k] = p < s1 ? __builtin_nontemporal_load(&mem[p]) : 0u;
                }
            }
#pragma unroll
            for (uint32_t k = 0; k < SS_LB; ++k) {
                const uint32_t p = s0 + 64 * (k0 + k) + lane;
                const uint32_t c = cv[k], m = mv[k];
                // pass 0 copied the words up to the sample's largest values (all below 2^18)
                if (p < s1 && (pass == 0 ? c > smc || m > smm : (c | m) >= RANK_MAX_VALUE)) miss = true;
                else if (p < s1) {
                    const uint32_t wc = BMC[c >> 5], wm = BMM[m >> 5];
                    if ((((wc >> (c & 31)) & (wm >> (m & 31))) & 1u) == 0u) {
                        miss = true;
                    } else {
                        const uint32_t rc = PRC[c >> 5] + (uint32_t)__popc(wc & ((1u << (c & 31)) - 1u));
                        const uint32_t rm = PRM[m >> 5] + (uint32_t)__popc(wm & ((1u << (m & 31)) - 1u));
                        const uint32_t hd = dc - 1u - rc, ld = dm - 1u - rm;
                        LD[p] = (uint8_t)ld;
                        ss_inc16(myrow, hd);
                        dvp[(k0 + k) >> 1] |= hd << (16u * ((k0 + k) & 1u));
                    }
                }
            }
        }
        if (__ballot(miss) && lane == 0) atomicOr(&NEXT[2], 1u);
        __syncthreads();
        if (NEXT[2] == 0u) return 0u;  // uniform
        __syncthreads();               // every thread has read NEXT[2] before pass 1 clears it
        return 1u;
    };
    uint32_t rr = samp ? rank_pass(0u) : 1u;
    if (rr == 1u) rr = rank_pass(1u);
    if (rr == 2u) return;  // (ss_generic ORed the scenario's values into a.rng)
    ss_offsets(WH, HS, HB, t, lane, w);
    const unsigned long long ck2 = SS_CLK();

    // ---- A1: stable scatter by hd, each wave over its own slice (digits from A0's registers) ----
#pragma unroll
    for (uint32_t k = 0; k < SS_CHUNKS; ++k) {
        const uint32_t p0 = s0 + 64 * k;
        if (p0 >= s1) break;  // wave-uniform
        const uint32_t p = p0 + lane;
        const bool valid = p < s1;
        const uint32_t d = (dvp[k >> 1] >> (16u * (k & 1u))) & 0xFFFFu;
        const uint64_t m = ss_match(d, valid, hbits);
        const uint32_t off = myrow[d];
        if (valid) {
            if ((m & lt) == 0) myrow[d] = (uint16_t)(off + __popcll(m));
            X[off + (uint32_t)__popcll(m & lt)] = (uint16_t)p;
        }
    }
    __syncthreads();
    const unsigned long long ck3 = SS_CLK();
    uint32_t big = 0;

    // ---- B: each hd bucket sorted by ld by one wave and written out ----
    while (true) {
        uint32_t d = 0;
        if (lane == 0) d = atomicAdd(NEXT, 1u);
        d = (uint32_t)__shfl((int)d, 0);
        if (d >= dc) break;
        const uint32_t lo = HS[d], hi = HB[d];
        if (lo == hi) continue;
        big = max(big, hi - lo);
        // the row is zeroed, counted with atomics, scanned and consumed by the same wave: the
        // fences keep those accesses in order (s_waitcnt lgkmcnt(0), no compiler reordering)
        reinterpret_cast<ss_u64a *>(myrow)[lane] = 0ull;  // 4 digits per lane
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        const uint32_t cv = CV[d];
        const uint32_t kbc = a.kpack ? (uint32_t)CB[d] << 21 : 0u;
        if (hi - lo <= 64 * SS_REG) {
            // the bucket in registers: count, scan, reorder X[lo, hi) in place, then write the
            // bucket's window of every output array coalesced
            uint32_t jv[SS_REG], lv[SS_REG];
#pragma unroll
            for (uint32_t k = 0; k < SS_REG; ++k) {
                const uint32_t p = lo + 64 * k + lane;
                jv[k] = p < hi ? X[p] : 0u;
                lv[k] = p < hi ? LD[jv[k]] : 0u;
                if (p < hi) ss_inc16(myrow, lv[k]);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            ss_row_scan(myrow, lane, lo);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll
            for (uint32_t k = 0; k < SS_REG; ++k) {
                if (lo + 64 * k >= hi) break;  // wave-uniform
                const bool valid = lo + 64 * k + lane < hi;
                const uint64_t m = ss_match(lv[k], valid, lbits);
                const uint32_t off = myrow[lv[k]];
                if (valid) {
                    if ((m & lt) == 0) myrow[lv[k]] = (uint16_t)(off + __popcll(m));
                    X[off + (uint32_t)__popcll(m & lt)] = (uint16_t)jv[k];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            for (uint32_t P = lo + lane; P < hi; P += 64) {
                const uint32_t j = X[P], l = LD[j];
                a.order[cb + P] = j;
                a.s_cpu[cb + P] = cv;
                a.s_mem[cb + P] = MV[l];
                a.s_idx[cb + P] = P | kbc | (a.kpack ? (uint32_t)MB[l] << 26 : 0u);
            }
        } else {  // a large bucket: the same stable order, scattered straight to HBM
#pragma unroll 4
            for (uint32_t p = lo + lane; p < hi; p += 64) ss_inc16(myrow, LD[X[p]]);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            ss_row_scan(myrow, lane, lo);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            for (uint32_t p0 = lo; p0 < hi; p0 += 64) {
                const uint32_t p = p0 + lane;
                const bool valid = p < hi;
                const uint32_t j = valid ? X[p] : 0u;
                const uint32_t l = valid ? LD[j] : 0u;
                const uint64_t m = ss_match(l, valid, lbits);
                const uint32_t off = myrow[l];
                if (valid) {
                    if ((m & lt) == 0) myrow[l] = (uint16_t)(off + __popcll(m));
                    const uint32_t P = off + (uint32_t)__popcll(m & lt);
                    a.order[cb + P] = j;
                    a.s_cpu[cb + P] = cv;
                    a.s_mem[cb + P] = MV[l];
                    a.s_idx[cb + P] = P | kbc | (a.kpack ? (uint32_t)MB[l] << 26 : 0u);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
#ifdef FP_PIPE_STATS
    const unsigned long long ck4 = SS_CLK();
    if (lane == 0) {
        atomicAdd(&g_sort_stats[4], ck4 - ck3);
        atomicMax(&g_sort_stats[6], (unsigned long long)big);
    }
    __syncthreads();
    if (t == 0) {
        const unsigned long long ck5 = SS_CLK();
        atomicAdd(&g_sort_stats[0], ck1 - ck0);
        atomicAdd(&g_sort_stats[1], ck2 - ck1);
        atomicAdd(&g_sort_stats[2], ck3 - ck2);
        atomicAdd(&g_sort_stats[3], ck5 - ck3);
        atomicAdd(&g_sort_stats[5], 1ull);
        atomicAdd(&g_sort_stats[7], ck5 - ck0);
    }
#else
    (void)ck0; (void)ck1; (void)ck2; (void)ck3; (void)big;
#endif
    // the batch's OR words (packed FFD records, fp_pipe_pk.h) from the value tables the digits rank
    // against: the scenario's own distinct values, or the sample's (a superset of them, and values
    // of the batch too) -- 2 x <= 256 LDS words by one wave, instead of registers kept live through
    // A0 (that spilled 162 VGPRs); at the end, where the fewest registers are live
    if (w == 0) {
        uint32_t oc = 0, om = 0;
        for (uint32_t i = lane; i < dc; i += 64) oc |= CV[i];
        for (uint32_t i = lane; i < dm; i += 64) om |= MV[i];
        for (int o = 32; o > 0; o >>= 1) {
            oc |= (uint32_t)__shfl_xor((int)oc, o);
            om |= (uint32_t)__shfl_xor((int)om, o);
        }
        if (lane == 0) {
            fp_or_new_bits(&a.rng[0], oc);
            fp_or_new_bits(&a.rng[1], om);
        }
    }
}

// T[0] = 0; T[1..31] spread evenly over the ascending distinct positive values v[0..d)
// (every value is a threshold when there are at most 31)
__device__ void value_thresholds(const uint32_t *v, uint32_t d, uint32_t *T) {
    while (d && v[0] == 0) { ++v; --d; }  // zero is T[0]
    T[0] = 0;
    for (int k = 1; k < FP_BUCKETS; ++k) {
        if (d == 0) { T[k] = 1; continue; }
        const uint64_t i = d <= (uint32_t)(FP_BUCKETS - 1) ? (uint64_t)(k - 1 < (int)d ? k - 1 : d - 1)
                                                             : (uint64_t)(k - 1) * (d - 1) / (FP_BUCKETS - 2);
        T[k] = v[i];
    }
}

// The pipeline's bucket thresholds, thr[0, K) cpu and [K, 2K) mem (thread 0: cpu, 1: mem): spread
// over the sample's distinct values when they are below 2^18 -- every bucket then spans about D / 31
// distinct values (config 4: 79 cpu and 256 mem values -> 2.5 and 8 per bucket; geometric steps
// spanned 9 and 43 at the top of the range, where most demands lie, and loose buckets cost exact
// checks that miss) -- else geometric from the smallest positive to the largest demand.  Any
// ascending choice with T[0] = 0 is exact: the thresholds only decide how tight the candidate masks
// are, so a sample of the batch sets them.
__global__ void k_thresholds(uint32_t *__restrict__ cnt, const uint32_t *__restrict__ cval,
                             const uint32_t *__restrict__ mval, uint32_t *__restrict__ thr) {
    const uint32_t d = threadIdx.x;
    if (d > 1) return;
    const bool ranks = cnt[CN_OVER] == 0;
    uint32_t T[FP_BUCKETS];
    if (ranks) {
        value_thresholds(d ? mval : cval, cnt[d ? CN_DM : CN_DC], T);
    } else {
        const uint32_t lo = cnt[d ? CN_MINM : CN_MINC], hi = cnt[d ? CN_MAXM : CN_MAXC];
        fp_thresholds(lo == 0xFFFFFFFFu ? 1u : lo, hi, T);
    }
    for (int k = 0; k < FP_BUCKETS; ++k) thr[d * FP_BUCKETS + k] = T[k];
}

// The sample's ranks as k_scen_sort's LDS image (pass 0 copies it): presence bitmaps [2][SR_W] u32,
// exclusive prefix counts [2][SR_W] u16, then per digit the mem and cpu values (digit d = rank
// dc-1-d) and their bucket ids.  Written only when the sample has <= 256 values per dimension, all
// below 2^18 (k_scen_sort tests the same counts).
__global__ __launch_bounds__(1024) void k_sort_image(const uint32_t *__restrict__ bm, const uint32_t *__restrict__ pre,
                                                     const uint32_t *__restrict__ val, const uint32_t *__restrict__ cnt,
                                                     const uint32_t *__restrict__ T, uint32_t kpack,
                                                     unsigned char *__restrict__ img) {
    const uint32_t dc = cnt[CN_DC], dm = cnt[CN_DM], t = threadIdx.x;
    if (cnt[CN_OVER] != 0u || dc - 1u >= SS_DIG || dm - 1u >= SS_DIG) return;
    uint32_t *ibm = reinterpret_cast<uint32_t *>(img);
    uint16_t *ipr = reinterpret_cast<uint16_t *>(ibm + 2 * SR_W);
    for (uint32_t i = t; i < 2 * SR_W; i += blockDim.x) {
        ibm[i] = bm[i];
        ipr[i] = (uint16_t)pre[i];
    }
    uint32_t *mv = reinterpret_cast<uint32_t *>(img + SR_BYTES), *cv = mv + SS_DIG;
    uint8_t *mb = reinterpret_cast<uint8_t *>(cv + SS_DIG), *cbk = mb + SS_DIG;
    if (t < SS_DIG) {
        const uint32_t c = t < dc ? val[dc - 1u - t] : 0u, m = t < dm ? val[RANK_MAX_VALUE + dm - 1u - t] : 0u;
        cv[t] = c;
        mv[t] = m;
        cbk[t] = kpack && t < dc ? (uint8_t)ss_bucket(T, c) : 0;
        mb[t] = kpack && t < dm ? (uint8_t)ss_bucket(T + FP_BUCKETS, m) : 0;
    }
}

}  // namespace

#ifdef FP_PIPE_STATS
extern "C" int fp_debug_sort_stats(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_stats), sizeof(unsigned long long) * 8) != hipSuccess)
        return FP_EDEVICE;
    if (reset) {
        static const unsigned long long zero[8] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sort_stats), zero, sizeof(zero)) != hipSuccess) return FP_EDEVICE;
    }
    return FP_OK;
}
#endif

static inline unsigned grid_for(size_t n, unsigned block) {
    size_t g = (n + block - 1) / block;
    if (g > 65535u * 4) g = 65535u * 4;
    return (unsigned)(g ? g : 1);
}

// Workspace bytes fp_dev_place_batch takes for S scenarios of C containers x N nodes
// (sort_tmp: the sorts' scratch share of it).
// scenarios whose values set the bucket thresholds (k_value_bitmap's sample)
constexpr uint32_t THR_SAMPLE = 8;

static int place_ws_need(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, size_t *need, size_t *sort_tmp_out) {
    hipStream_t st = c->stream;
    const size_t SC = (size_t)S * C;
    // the radix path sorts full-width u64 keys: device-wide for one scenario, segmented for several
    size_t sort_tmp = 0, t = 0;
    FP_HIP(rocprim::radix_sort_pairs(nullptr, t, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                     (uint32_t *)nullptr, SC, 0, 64, st));
    sort_tmp = t;
    FP_HIP(rocprim::segmented_radix_sort_pairs(nullptr, t, (uint64_t *)nullptr,
                                               (uint64_t *)nullptr, (uint32_t *)nullptr,
                                               (uint32_t *)nullptr, (unsigned)SC, S,
                                               (uint32_t *)nullptr, (uint32_t *)nullptr, 0, 64, st));
    sort_tmp = t > sort_tmp ? t : sort_tmp;
    const size_t pipe_ws = fp_pipe_ws_bytes(c, S, C, N);
    if (pipe_ws == 0) return FP_EOVERFLOW;
    const size_t rank_ws = 2 * (2 * RANK_WORDS * 4 + RANK_MAX_VALUE * 4) + CN_WORDS * 4 + 2 * FP_BUCKETS * 4 + 3 * 256
                           + SS_IMG_BYTES + 256;
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
    c->last_rng = nullptr;
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
    // rank tables: bitmaps + prefix counts [2][RANK_WORDS] each, value tables, counts / bounds /
    // eligibility (CN_*), thresholds [2][FP_BUCKETS] -- all device-resident, nothing is read back
    uint32_t *rbm = (uint32_t *)fp_ws_take(c, 2 * RANK_WORDS * 4);
    uint32_t *rpre = (uint32_t *)fp_ws_take(c, 2 * RANK_WORDS * 4);
    uint32_t *rval = (uint32_t *)fp_ws_take(c, 2 * RANK_MAX_VALUE * 4);
    uint32_t *rcnt = (uint32_t *)fp_ws_take(c, CN_WORDS * 4);
    uint32_t *thr = (uint32_t *)fp_ws_take(c, 2 * FP_BUCKETS * 4);
    unsigned char *simg = (unsigned char *)fp_ws_take(c, SS_IMG_BYTES);
    if (!keys_in || !keys_out || !vals_in || !vals_out || !offs || !tmp || !rbm || !rpre || !rval || !rcnt || !thr ||
        !simg)
        return FP_ENOMEM;
    c->last_rng = rcnt + CN_ORC;

    // ---- 1-2: the bucket thresholds (device), from the distinct values and bounds of a sample:
    // the first THR_SAMPLE scenarios (any ascending thresholds with T[0] = 0 are exact; they only
    // set how tight the pipeline's candidate masks are) ----
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_SORT, &ev);
    FP_HIP(hipMemsetAsync(rbm, 0, 2 * RANK_WORDS * 4, st));
    FP_HIP(hipMemsetAsync(rcnt, 0, CN_WORDS * 4, st));
    FP_HIP(hipMemsetAsync(rcnt + CN_MINC, 0xFF, 8, st));  // the minima start at 0xFFFFFFFF
    {
        const size_t n = (size_t)(S < THR_SAMPLE ? S : THR_SAMPLE) * C;
        unsigned gb = grid_for((n + 3) / 4, 256);
        if (gb > 1024) gb = 1024;  // each block merges its bitmaps once
        FP_HIP(hipFuncSetAttribute((const void *)k_value_bitmap, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(2 * RANK_WORDS * 4)));
        k_value_bitmap<<<gb, 256, 2 * RANK_WORDS * 4, st>>>(b->cpu_m, b->mem_mib, n, rbm, rbm + RANK_WORDS, rcnt);
        FP_HIP(hipGetLastError());
        k_rank_tables<<<2, 1024, 0, st>>>(rbm, rbm + RANK_WORDS, RANK_WORDS, RANK_WORDS, rpre, rpre + RANK_WORDS, rval,
                                          rval + RANK_MAX_VALUE, rcnt);
        FP_HIP(hipGetLastError());
        k_thresholds<<<1, 64, 0, st>>>(rcnt, rval, rval + RANK_MAX_VALUE, thr);
        FP_HIP(hipGetLastError());
    }
    // ---- 3a: per-scenario LDS sort (scenarios of at most ~50k containers; host-known).  A scenario
    // without dense ranks of <= 256 values per dimension takes k_scen_sort's generic fallback,
    // chosen in its workgroup.  FP_OPT_SCEN_SORT = 0 keeps the radix path. ----
    if (ss_lds_bytes(C) <= SS_LDS_CAP && C <= SS_WAVES * SS_CHUNKS * 64 && fp_opt(c, FP_OPT_SCEN_SORT, 1) != 0) {
        ScenSortArgs sa;
        sa.C = C; sa.kpack = fp_pipe_kpack(c, C);
        sa.cpu = b->cpu_m; sa.mem = b->mem_mib;
        fp_pipe_soa soa;
        if (int rs = fp_pipe_soa_take(c, SC, &soa)) return rs;
        sa.order = vals_out; sa.s_cpu = soa.s_cpu; sa.s_mem = soa.s_mem; sa.s_idx = soa.s_idx;
        sa.T = thr;
        sa.scnt = rcnt;
        sa.rng = rcnt + CN_ORC;
        sa.simg = simg;
        k_sort_image<<<1, 1024, 0, st>>>(rbm, rpre, rval, rcnt, thr, sa.kpack, simg);
        FP_HIP(hipGetLastError());
        const size_t lds = ss_lds_bytes(C);
        FP_HIP(hipFuncSetAttribute((const void *)k_scen_sort, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        k_scen_sort<<<S, 1024, lds, st>>>(sa);
        FP_HIP(hipGetLastError());
        fp_prof_end(c, FP_K_SORT, ev);
        return fp_pipe_launch(c, S, C, N, b->scen_base, vals_out, nullptr, 4, 0, 0, 0, rval, rval + RANK_MAX_VALUE, b,
                              thr, &soa, rcnt + CN_ORC);
    }
    // ---- 3b: radix path: key = (~cpu << 32 | ~mem), value = the container's index; a stable
    // radix sort over all 64 bits gives (cpu desc, mem desc, index asc) without knowing the key
    // range on the host (FP_OPT_SEGSORT no longer changes anything: several scenarios are always
    // sorted as segments, one scenario device-wide) ----
    const uint64_t full = 0xFFFFFFFFull;
    k_make_keys<<<grid_for(SC, 256), 256, 0, st>>>(b->cpu_m, b->mem_mib, SC, C, keys_in, vals_in, rcnt + CN_ORC);
    FP_HIP(hipGetLastError());
    if (S == 1) {
        FP_HIP(rocprim::radix_sort_pairs(tmp, sort_tmp, keys_in, keys_out, vals_in, vals_out, SC, 0, 64, st));
    } else {
        k_seg_offsets<<<(S + 1 + 255) / 256, 256, 0, st>>>(S, C, offs);
        FP_HIP(hipGetLastError());
        FP_HIP(rocprim::segmented_radix_sort_pairs(tmp, sort_tmp, keys_in, keys_out, vals_in, vals_out, (unsigned)SC,
                                                   S, offs, offs + 1, 0, 64, st));
    }
    fp_prof_end(c, FP_K_SORT, ev);
    // ---- 4-5: placement + cost ----
    return fp_pipe_launch(c, S, C, N, b->scen_base, vals_out, keys_out, 8, 32, full, full, nullptr, nullptr, b, thr,
                          nullptr, rcnt + CN_ORC);
}

extern "C" int fp_ctx_place_path(fp_ctx *c, uint32_t *out3) {
    if (!c || !out3) return FP_EINVAL;
    out3[0] = out3[1] = out3[2] = 0u;
    if (!c->last_rng) return FP_OK;
    FP_HIP(hipSetDevice(c->device));
    FP_HIP(hipStreamSynchronize(c->stream));
    FP_HIP(hipMemcpy(out3, c->last_rng, 12, hipMemcpyDeviceToHost));
    return FP_OK;
}

extern "C" int fp_dev_argmin_cost(fp_ctx *c, const uint64_t *cost, uint32_t n, uint32_t *best) {
    if (!c || !cost || !best || n == 0) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    k_argmin_cost<<<1, 1024, 0, c->stream>>>(cost, n, best);
    return fp_dev_done(c, hipGetLastError() == hipSuccess ? FP_OK : FP_EDEVICE);
}
