// fp_order.hip -- stage 1: start ordering.
//
//  * fp_dev_legacy_order: crates/fleetflow-container/src/engine.rs:67-85 as a stable
//    two-bucket partition (has_deps == 0 first, each bucket in input order),
//    computed with wavefront ballots + a block-offset scan.
//  * fp_dev_levelize: SPEC.md 2.2, Kahn over the reversed CSR, asynchronous by default
//    (k_lvl_async: a persistent grid on sharded work queues, no per-level launch;
//    DESIGN.md 4.4), level-synchronous with FP_OPT_LEVELIZE_SYNC (one k_expand
//    launch per level).  level(v) = max(has_deps(v), max_{d->v} level(d)+1) is unique,
//    so neither schedule (nor the atomic order inside it) can change the result.
#include "fp_internal.h"
#include "fp_small.h"
#include <rocprim/device/device_radix_sort.hpp>
#include <stdlib.h>
#include <string.h>

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 4;                  // items per thread per block
constexpr int kSpan = kBlock * kItems;     // items per block

// Count has_deps == 0 per block.
__global__ __launch_bounds__(kBlock) void k_part_count(const uint8_t *__restrict__ hd, uint32_t n,
                                                       uint32_t *__restrict__ blk_zero) {
    __shared__ uint32_t wsum[kBlock / 64];
    uint32_t z = 0;
    const size_t base = (size_t)blockIdx.x * kSpan;
    for (int it = 0; it < kItems; ++it) {
        const size_t i = base + (size_t)it * kBlock + threadIdx.x;
        z += (i < n && hd[i] == 0) ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) z += __shfl_xor(z, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = z;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += wsum[w];
        blk_zero[blockIdx.x] = t;
    }
}

// The whole partition in one launch for n <= 1024 (a stage of a fleet.kdl: config 1), one thread
// per vertex: the three kernels below cost a launch each.
__global__ __launch_bounds__(1024) void k_part_small(const uint8_t *__restrict__ hd, uint32_t n,
                                                     uint32_t *__restrict__ perm) {
    __shared__ uint32_t wsum[16];
    const uint32_t i = threadIdx.x, lane = i & 63, w = i >> 6;
    const bool z = i < n && hd[i] == 0;
    const uint64_t m = __ballot(z);
    if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t woff = 0, tot = 0;
    for (uint32_t q = 0; q < 16; ++q) {
        woff += q < w ? wsum[q] : 0u;
        tot += wsum[q];
    }
    if (i < n) {
        const uint32_t zb = woff + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));  // zeros before i
        perm[z ? zb : tot + i - zb] = i;
    }
}

// Exclusive scan of block counts by one block; writes total to blk_off[nb].
__global__ __launch_bounds__(1024) void k_part_scan(const uint32_t *__restrict__ blk_zero,
                                                    uint32_t nb, uint32_t *__restrict__ blk_off) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t v = b < nb ? blk_zero[b] : 0u;
        uint32_t x = v;  // inclusive wave scan
        const uint32_t lane = threadIdx.x & 63;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t woff = 0;
        for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) woff += wsum[w];
        const uint32_t c0 = carry;
        if (b < nb) blk_off[b] = c0 + woff + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = c0 + woff + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) blk_off[nb] = carry;
}

__global__ __launch_bounds__(kBlock) void k_part_scatter(const uint8_t *__restrict__ hd, uint32_t n,
                                                         const uint32_t *__restrict__ blk_off,
                                                         uint32_t nb, uint32_t *__restrict__ perm) {
    __shared__ uint32_t wsum[kBlock / 64];
    const uint32_t total_zero = blk_off[nb];
    uint32_t zeros_before = blk_off[blockIdx.x];  // block-uniform running count
    const size_t base = (size_t)blockIdx.x * kSpan;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int it = 0; it < kItems; ++it) {
        const size_t i = base + (size_t)it * kBlock + threadIdx.x;
        const bool z = i < n && hd[i] == 0;
        const uint64_t m = __ballot(z);
        const uint32_t wrank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t woff = 0, tot = 0;
        for (int q = 0; q < kBlock / 64; ++q) {
            if (q < (int)w) woff += wsum[q];
            tot += wsum[q];
        }
        if (i < n) {
            const uint32_t zb = zeros_before + woff + wrank;  // zeros strictly before i
            perm[z ? zb : total_zero + (uint32_t)i - zb] = (uint32_t)i;
        }
        zeros_before += tot;
        __syncthreads();
    }
}

// ---- levelize -----------------------------------------------------------------
// A corrupt CSR raises FP_ECORRUPT in the (sticky) error word AND this call's own `bad` word:
// every later kernel of the call reads `bad` and does nothing, so no expansion runs on an
// invalid graph and the host never waits for the check (fp_dev_levelize stays asynchronous).
__device__ __forceinline__ void lv_corrupt(uint32_t *err, uint32_t *bad) {
    atomicMax(err, (uint32_t)(-FP_ECORRUPT));
    atomicOr(bad, 1u);
}

__global__ void k_check_csr(const uint32_t *__restrict__ row_ptr, uint32_t V, uint32_t E,
                            uint32_t *__restrict__ err, uint32_t *__restrict__ bad) {
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) {
        if (row_ptr[v + 1] < row_ptr[v]) lv_corrupt(err, bad);
    }
    if (v == 0 && (row_ptr[0] != 0 || row_ptr[V] != E)) lv_corrupt(err, bad);
}

__global__ void k_indeg(const uint32_t *__restrict__ col, uint32_t E, uint32_t V,
                        uint32_t *__restrict__ indeg, uint32_t *__restrict__ err, uint32_t *__restrict__ bad) {
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = col[e];
        if (v >= V) lv_corrupt(err, bad);
        else atomicAdd(&indeg[v], 1u);
    }
}

__global__ void k_lvl_init(const uint8_t *__restrict__ hd, const uint32_t *__restrict__ indeg,
                           uint32_t V, uint32_t *__restrict__ level,
                           uint32_t *__restrict__ frontier, uint32_t *__restrict__ fcount) {
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = v < V;
    const bool src = in && indeg[v] == 0;
    if (in) level[v] = hd[v] ? 1u : 0u;
    // wave-aggregated push
    const uint64_t m = __ballot(src);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(fcount, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    if (src) frontier[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)v;
}

// One thread per frontier vertex; relax its out-edges.  Level L's frontier size
// is read from cnt[L] on the device and level L+1's is counted into cnt[L+1], so
// the host enqueues levels without reading anything back (no per-level sync).
__global__ void k_expand(const uint32_t *__restrict__ frontier, const uint32_t *__restrict__ cnt_l,
                         const uint32_t *__restrict__ row_ptr, const uint32_t *__restrict__ col,
                         uint32_t *__restrict__ level, uint32_t *__restrict__ indeg,
                         uint32_t *__restrict__ next, uint32_t *__restrict__ cnt_next) {
    const uint32_t fsize = *cnt_l;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < fsize;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t u = frontier[i];
        const uint32_t lu1 = level[u] + 1u;
        const uint32_t e1 = row_ptr[u + 1];
        for (uint32_t e = row_ptr[u]; e < e1; ++e) {
            const uint32_t v = col[e];
            atomicMax(&level[v], lu1);
            if (atomicSub(&indeg[v], 1u) == 1u) next[atomicAdd(cnt_next, 1u)] = v;
        }
    }
}

__global__ void k_lvl_final(const uint32_t *__restrict__ indeg, uint32_t V, uint32_t cyc_key,
                            uint32_t *__restrict__ level, uint32_t *__restrict__ keys, uint32_t *__restrict__ vals,
                            uint32_t *__restrict__ ncyc, uint32_t *__restrict__ ck) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *ck = cyc_key;
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool cyc = v < V && indeg[v] != 0;
    if (v < V) {
        if (cyc) level[v] = FP_NONE;
        keys[v] = cyc ? cyc_key : level[v];
        vals[v] = (uint32_t)v;
    }
    const uint64_t m = __ballot(cyc);
    if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd(ncyc, (uint32_t)__popcll(m));
}

// ---- asynchronous levelizer (no level barriers) -------------------------------------
// A persistent grid works a sharded queue of ready vertices.  Per vertex v a packed
// state word holds (max level seen << 32 | parents still to come); a parent u relaxes
// the edge u -> v with one CAS (level max(., level(u)+1), count - 1).  The CAS that
// takes the count to zero owns v: its level is final (every parent's update landed
// in the same word before).  The owner continues with its first ready child in the
// same lane (a chain never touches the queue) and pushes the others.  So a chain of
// depth D costs D dependent (row_ptr, col, CAS) round trips, not D kernel launches.
// Termination: done[] counts queue items whose lane (and continuation chain) has
// finished, tail[] counts pushed items; done == tail means nothing is in flight and
// nothing can be pushed again.  One monitor lane checks it and raises `fin`.
#ifndef LVL_SHARDS
#define LVL_SHARDS 8
#endif
// queues (blocks b and b+8 share an XCD); 16 queues: config 5 -1 %, 32: +2 % (profiles/r07n_lvl_ab.txt)
constexpr uint32_t kShards = LVL_SHARDS;
constexpr uint32_t kCtlStride = 32;       // u32 words between counters (128 B lines)
constexpr uint32_t kFinWord = 3 * kShards * kCtlStride, kAbortWord = kFinWord + kCtlStride;
constexpr uint32_t kMaxLevelWord = kAbortWord + kCtlStride;  // ctl word: the largest level the schedule wrote
constexpr uint64_t kQEmpty = ~0ull;
// edges left at which the wave expands a vertex together, and edges a lane relaxes per round
// (config 5: 16 / 1 0.775 ms; cooperative at 8 0.823, at 32 0.779; 2 edges per lane 0.877;
// profiles/r04aa_lvl_tuning_ab.txt)
#ifndef LVL_COOP_EDGES  // round 6: 8 / 32 edges 0.670-0.674 / 0.621-0.626 against 0.623-0.626 ms; 16 queues
#define LVL_COOP_EDGES 16  // 0.633-0.638 (profiles/r08p_lvl_ab.txt)
#endif
constexpr uint32_t kCoopEdges = LVL_COOP_EDGES;
constexpr uint32_t kLaneEdges = 1;
// levels a lane may jump per round along only-parent first edges: 4 (config 5 0.84 ms; 6 hops 0.86, 8 hops
// 0.92 -- more records to build and load per round, profiles/r04m_lvl_hops_ab.txt; round 6 at 16-B queue
// entries: 4 / 6 / 8 hops 0.663-0.665 / 0.664-0.665 / 0.738 ms, profiles/r07p_lvl_ab.txt; final tree:
// 2 / 3 / 5 hops 0.677-0.679 / 0.631-0.635 / 0.626-0.632 against 0.622-0.624 ms, profiles/r09l_lvl_ab.txt)
#ifndef LVL_HOPS
#define LVL_HOPS 4
#endif
constexpr uint32_t kHops = LVL_HOPS;
constexpr uint32_t kPush = kLaneEdges + kHops;  // queue entries a lane may push per round
// one-wave blocks of the persistent grid: 8 waves per CU (config 5: 2048 0.78 ms, 512 0.84, 4096 0.79,
// 8192 0.81, 256 0.92; profiles/r04v_lvl_grid_ab.txt) -- a wave round lasts as long as its slowest
// lane, so spreading the items over more waves shortens the rounds of the lanes on the long chains,
// until idle waves' queue polls start to cost more
#ifndef LVL_BLOCKS  // round 6 at 16-B entries: 1024 / 1536 / 3072 blocks 0.647-0.650 / 0.633 / 0.636-0.640
#define LVL_BLOCKS 2048  // against 0.624-0.629 ms (profiles/r08o_lvl_ab.txt)
#endif
constexpr uint32_t kAsyncBlocks = LVL_BLOCKS;
constexpr uint32_t kInitClaims = kAsyncBlocks / kShards * 64u;  // slots per shard claimed at the start
#ifndef LVL_SLEEP_LONG
#define LVL_SLEEP_LONG 8  // s_sleep of an idle wave after LVL_IDLE_SPIN short (s_sleep 1) rounds (2 / 32: +-1 %, r07k)
#endif
#ifndef LVL_IDLE_SPIN  // final tree: 4 / 64 short rounds, long sleep 4: all within +-0.5 % (profiles/r09n_lvl_ab.txt)
#define LVL_IDLE_SPIN 16
#endif

// ctl layout (u32 index, S = kShards): head[s] = s*32, tail[s] = (S+s)*32, done[s] = (2S+s)*32,
// fin = 3S*32, abort = (3S+1)*32, maxlvl = (3S+2)*32
constexpr uint32_t kCtlWords = kMaxLevelWord + kCtlStride;

// Diagnostics build only (-DFP_LVL_TRACE, tools/lvl_trace.py): the first time each level is
// written by k_lvl_async (s_memrealtime, 100 MHz), [4094] the earliest wave start, [4095] the last
// wave exit.  Read back with fp_debug_lvl_trace.
#ifdef FP_LVL_TRACE
__device__ unsigned long long g_lvl_trace[4096];
// (a lane keeps the deepest level it wrote in a round with its time; the next round loads that
// level's word beside its records and lowers it only when this lane was first, so the hot words
// of the last levels see few atomics -- an atomic per write slowed config 5 from 0.5 to 2.3 ms)
#define LVL_TR(L)                                                                                        \
    do {                                                                                                 \
        if ((L) > my_max && (trL == FP_NONE || (L) > trL)) {                                             \
            trL = min((uint32_t)(L), 4093u);                                                             \
            trT = __builtin_amdgcn_s_memrealtime();                                                      \
        }                                                                                                \
    } while (0)
extern "C" __attribute__((visibility("default"))) int fp_debug_lvl_trace(uint64_t *out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lvl_trace), sizeof(g_lvl_trace)) == hipSuccess ? 0 : -1;
}
#else
#define LVL_TR(L) ((void)0)
#endif

__device__ __forceinline__ uint64_t ag_ld64(const uint64_t *p) {
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ag_ld32(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ag_rmw_rd(uint32_t *p) {  // coherent read (an RMW)
    return __hip_atomic_fetch_add(p, 0u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

// Sources (in-degree 0) with out-edges go to the queues; every other vertex starts
// at level NONE (a source without out-edges is final here).
// One 16-B record per CSR edge: the child, the child's own edge range, and whether this edge
// is the child's only in-edge.  A chain hop then costs one load round trip: the record of the
// continuation's first edge names the next vertex AND where its edges are, and a child whose
// only parent is the expanding vertex is ready without an atomic (its level is the parent's
// + 1 >= has_deps; nothing else ever touches its state word).  Round 2 paid three: col[e],
// then row_ptr[w] beside the CAS on state[w], then the next col.
// Round 3 adds kHops - 1 records per edge, the hops after it along first edges: rec2[h][e] is
// the h-th vertex reached from the edge's child by always taking the first edge (that vertex,
// its edge range, whether the edge into it is its only in-edge).  When the child w is ready with
// its only parent and its first dependent w2 has w as its only parent (and so on), a lane jumps
// several levels in one round trip: each level is the previous + 1, no atomic on any of them,
// and the rest of each passed vertex's edges goes to the queue as a partial item.  A chain of
// depth D takes ~D / kHops rounds.  (Two levels per round: config-5 levelize 1.51 -> 1.13 ms.)

// ---- the async path's set-up in four launches (round 5; was 12 launches and memsets) -----------
// The work queues (kShards x V 16-B entries, 128 MB at config 5) live in a context buffer of their own
// (fp_ctx::lvl_q): k_lvl_async resets every slot it consumes, so a levelization that finishes
// cleanly leaves them empty and marks the buffer clean (qflag = kQClean); the next call fills them
// with kQEmpty only when the flag says otherwise (a fresh buffer, an aborted or corrupt call).
constexpr uint32_t kQClean = 0x600Du;

// in-degrees, the call's counters, the control words and the caller's n_cycle word zeroed; the
// queues emptied when dirty
__global__ void k_lvl_zero(uint32_t V, uint32_t *__restrict__ indeg, uint32_t *__restrict__ ncyc,
                           uint32_t *__restrict__ actl, uint32_t *__restrict__ ncyc_out, uint4 *__restrict__ Q4,
                           size_t q4, const uint32_t *__restrict__ qflag) {
    const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    for (size_t i = i0; i < V; i += st) indeg[i] = 0u;
    if (i0 < 16) ncyc[i0] = 0u;
    // the claim heads start past the slots every wave holds from its start (k_lvl_async)
    for (size_t i = i0; i < kCtlWords; i += st)
        actl[i] = i < kShards * kCtlStride && i % kCtlStride == 0 ? kInitClaims : 0u;
    if (i0 == 0 && ncyc_out) *ncyc_out = 0u;
    if (*qflag != kQClean)
        for (size_t i = i0; i < q4; i += st) Q4[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
}

// the CSR check (k_check_csr's conditions) and the in-degrees (k_indeg) in one pass; marks the
// queues dirty until k_lvl_async finishes cleanly
__global__ void k_indeg_check(const uint32_t *__restrict__ row_ptr, const uint32_t *__restrict__ col, uint32_t V,
                              uint32_t E, uint32_t *__restrict__ indeg, uint32_t *__restrict__ err,
                              uint32_t *__restrict__ bad, uint32_t *__restrict__ qflag) {
    const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    if (i0 == 0) {
        *qflag = 0u;
        if (row_ptr[0] != 0 || row_ptr[V] != E) lv_corrupt(err, bad);
    }
    const size_t n = V > E ? V : E;
    for (size_t i = i0; i < n; i += st) {
        if (i < V && row_ptr[i + 1] < row_ptr[i]) lv_corrupt(err, bad);
        if (i < E) {
            const uint32_t v = col[i];
            if (v >= V) lv_corrupt(err, bad);
            else atomicAdd(&indeg[v], 1u);
        }
    }
}

// The in-degrees without global atomics (round 5; FP_OPT_INDEG_BIN = 0 keeps k_indeg_check).
// k_indeg_check's 1.75M atomicAdds on random words run at the memory side, one request per lane
// (config 5: 67 us).  Here the edges are binned by child range instead: k_indeg_bin sorts each
// 4096-edge slice by bucket (child >> shift, at most kBinMaxB buckets) in LDS and writes it back in
// place with the bucket starts (transposed: offt[b * nwg + slice], row B = the slice's total);
// k_indeg_hist counts one bucket's children in LDS from every slice's run and stores its range's
// in-degrees coalesced, beside the row_ptr checks and a 16-B vertex record (its edge range, whether
// it has one parent) that k_lvl_prep's edge records then take in one random load instead of two lines.
constexpr uint32_t kBinT = 256, kBinPer = 16, kBinSlice = kBinT * kBinPer, kBinMaxB = 1024;
constexpr uint32_t kBinMinShift = 12, kBinMaxShift = 14;  // bucket ranges 4096 .. 16384 vertices
constexpr uint32_t kHistT = 1024;

__global__ __launch_bounds__(kBinT) void k_indeg_bin(const uint32_t *__restrict__ col, uint32_t V, uint32_t E,
                                                     uint32_t shift, uint32_t B, uint32_t nwg,
                                                     uint32_t *__restrict__ binned, uint32_t *__restrict__ offt,
                                                     uint32_t *__restrict__ err, uint32_t *__restrict__ bad,
                                                     uint32_t *__restrict__ qflag) {
    __shared__ uint32_t cnt[kBinMaxB + 1];
    __shared__ uint32_t wsum[kBinT / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const size_t e0 = (size_t)blockIdx.x * kBinSlice;
    if (blockIdx.x == 0 && t == 0) *qflag = 0u;
    for (uint32_t b = t; b < 4 * kBinT; b += kBinT) cnt[b] = 0u;
    __syncthreads();
    uint32_t v[kBinPer], r[kBinPer];
#pragma unroll
    for (uint32_t k = 0; k < kBinPer; ++k) {
        const size_t i = e0 + k * kBinT + t;
        v[k] = i < E ? col[i] : ~0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kBinPer; ++k) {
        const size_t i = e0 + k * kBinT + t;
        if (i < E && v[k] >= V) lv_corrupt(err, bad);
        if (v[k] < V) r[k] = atomicAdd(&cnt[v[k] >> shift], 1u);
    }
    __syncthreads();
    // exclusive scan of the bucket counts: thread t holds buckets [4t, 4t + 4)
    uint32_t c4[4], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        c4[j] = cnt[4 * t + j];
        s += c4[j];
    }
    uint32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        if ((int)lane >= o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t run = inc - s;
    for (uint32_t w = 0; w < wv; ++w) run += wsum[w];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        cnt[4 * t + j] = run;
        run += c4[j];
    }
    if (t == kBinT - 1) cnt[B] = run;  // the slice's total (buckets >= B count nothing)
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kBinPer; ++k)
        if (v[k] < V) binned[e0 + cnt[v[k] >> shift] + r[k]] = v[k];
    for (uint32_t b = t; b <= B; b += kBinT) offt[(size_t)b * nwg + blockIdx.x] = cnt[b];
}

// one workgroup per bucket: split = threads per slice run (a power of two, nwg * split <= kHistT
// where the slices are few), each thread four loads in flight
__global__ __launch_bounds__(kHistT) void k_indeg_hist(const uint32_t *__restrict__ binned,
                                                       const uint32_t *__restrict__ offt, uint32_t nwg,
                                                       uint32_t split, uint32_t shift, uint32_t V, uint32_t E,
                                                       const uint32_t *__restrict__ row_ptr,
                                                       uint32_t *__restrict__ indeg, uint4 *__restrict__ vrec,
                                                       uint32_t *__restrict__ err, uint32_t *__restrict__ bad) {
    extern __shared__ uint32_t h[];
    const uint32_t t = threadIdx.x, b = blockIdx.x;
    const uint32_t v0 = b << shift, n = min(V - v0, 1u << shift);
    for (uint32_t i = t; i < n; i += kHistT) h[i] = 0u;
    __syncthreads();
    const uint32_t part = t & (split - 1);
    for (uint32_t sl = t / split; sl < nwg; sl += kHistT / split) {
        const uint32_t *p = binned + (size_t)sl * kBinSlice;
        const uint32_t a = offt[(size_t)b * nwg + sl] + part, z = offt[(size_t)(b + 1) * nwg + sl];
        for (uint32_t i = a; i < z; i += 4 * split) {
            uint32_t x[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) x[k] = i + k * split < z ? p[i + k * split] : ~0u;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k)
                if (x[k] != ~0u) atomicAdd(&h[x[k] - v0], 1u);
        }
    }
    __syncthreads();
    if (b == 0 && t == 0 && (row_ptr[0] != 0 || row_ptr[V] != E)) lv_corrupt(err, bad);
#pragma unroll 4
    for (uint32_t i = t; i < n; i += kHistT) {
        const uint32_t v = v0 + i, r0 = row_ptr[v], r1 = row_ptr[v + 1], d = h[i];
        indeg[v] = d;
        if (r1 < r0) lv_corrupt(err, bad);
        vrec[v] = make_uint4(r0, r1, d == 1u ? 1u : 0u, 0u);  // k_lvl_prep's edge records: one gather
    }
}

// The vertex states and the source queue items (blocks [0, vblocks): one vertex per thread) beside
// the edge records (the other blocks, grid-stride over the edges) in one launch
__global__ void k_lvl_prep(const uint8_t *__restrict__ hd, const uint32_t *__restrict__ indeg,
                           const uint32_t *__restrict__ row_ptr, const uint32_t *__restrict__ col, uint32_t V,
                           uint32_t E, uint32_t vblocks, uint32_t *__restrict__ level, uint64_t *__restrict__ state,
                           uint4 *__restrict__ Q, uint32_t *__restrict__ ctl, uint4 *__restrict__ rec,
                           const uint4 *__restrict__ vrec, const uint32_t *__restrict__ bad) {
    if (*bad) return;
    if (blockIdx.x < vblocks) {
        const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
        const bool in = v < V;
        uint32_t l0 = 0, deg = 0;
        bool src = false;
        if (in) {
            l0 = hd[v] ? 1u : 0u;
            deg = row_ptr[v + 1] - row_ptr[v];
            src = indeg[v] == 0;
            state[v] = ((uint64_t)l0 << 32) | indeg[v];
            level[v] = src && deg == 0 ? l0 : FP_NONE;
        }
        const bool push = src && deg != 0;
        const uint64_t m = __ballot(push);
        if (!m) return;
        const uint32_t lane = threadIdx.x & 63, leader = (uint32_t)__builtin_ctzll(m);
        const uint32_t sh = (uint32_t)((v >> 6) % kShards);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&ctl[(kShards + sh) * kCtlStride], (uint32_t)__popcll(m));
        base = __shfl(base, (int)leader);
        if (push)  // a 16-B queue entry (k_lvl_async): (level << 32 | v, first edge << 32 | end edge)
            Q[(size_t)sh * V + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] =
                make_uint4((uint32_t)v, l0, row_ptr[v + 1], row_ptr[v]);
        return;
    }
    const size_t st = (size_t)(gridDim.x - vblocks) * blockDim.x;
    for (size_t e = (size_t)(blockIdx.x - vblocks) * blockDim.x + threadIdx.x; e < E; e += st) {
        const uint32_t w = col[e];  // < V: k_indeg_check / k_indeg_bin raised `bad` otherwise
        if (vrec) {
            const uint4 r = vrec[w];
            rec[e] = make_uint4(w, r.x, r.y, r.z);
        } else {
            rec[e] = make_uint4(w, row_ptr[w], row_ptr[w + 1], indeg[w] == 1u ? 1u : 0u);
        }
    }
}

// The kernel after k_lvl_prep: the kHops - 1 hops of every edge whose child has it as its only
// in-edge, by chasing the finished records along first edges (hop h + 1 of e = the record of the
// first edge of hop h's vertex, kept while every edge on the way is its child's only in-edge).
// k_lvl_async reads an edge's hops only when the edge itself is an only-parent edge (rec.w), so the
// hops of the other edges are left unwritten.  (Chasing col / row_ptr / indeg inside k_lvl_prep
// instead: 0.121 ms against 0.07, profiles/r05b_lvl_kernel_stats.csv.)
__global__ void k_edge_hops(uint32_t E, const uint4 *__restrict__ rec, uint4 *__restrict__ rec2,
                            const uint32_t *__restrict__ bad) {
    if (*bad) return;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (size_t)gridDim.x * blockDim.x) {
        uint4 cur = rec[e];
        if (cur.w == 0u) continue;
        bool ok = true;
#pragma unroll
        for (uint32_t h = 0; h + 1 < kHops; ++h) {
            uint4 nx = make_uint4(0u, 0u, 0u, 0u);
            if (ok && cur.z > cur.y && cur.y < E) {
                const uint4 f = rec[cur.y];
                if (f.w != 0u) nx = f;
            }
            rec2[(size_t)h * E + e] = nx;
            ok = nx.w != 0u;
            cur = nx;
        }
    }
}

// Queue entries are 16 B: lo = (level << 32) | vertex, hi = (first edge << 32) | end edge, so a lane
// that claims an item has its edge range with it (no row_ptr round trip).  Only vertices with edges
// left are pushed (a ready child without out-edges is final where it becomes ready), so a valid hi
// has first edge < end edge <= E and is never the empty marker; an entry is taken only when both
// halves are valid (the producer's two stores may land in either order).
struct QEnt {
    uint64_t lo, hi;
};
__device__ __forceinline__ QEnt q_ent(uint32_t v, uint32_t lvl, uint32_t e0, uint32_t e1) {
    return QEnt{((uint64_t)lvl << 32) | v, ((uint64_t)e0 << 32) | e1};
}
__device__ __forceinline__ void q_store(uint64_t *slot2, const QEnt &x) {
    __hip_atomic_store(slot2 + 1, x.hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(slot2, x.lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The pushes of one round: entries, per-lane offsets, the target queue, the reservation's result
// (lane 0) and the items the round finished (their done count follows the entries' stores).
struct PushSet {
    bool pend[kPush];
    uint32_t pofs[kPush];
    QEnt pent[kPush];
    uint32_t tot, ps, pbase, ndone;
};

__global__ __launch_bounds__(64) void k_lvl_async(const uint4 *__restrict__ erec, const uint4 *__restrict__ erec2,
                                                  uint32_t E, uint32_t V, uint64_t *__restrict__ state,
                                                  uint64_t *__restrict__ Q, uint32_t *__restrict__ ctl,
                                                  uint32_t *__restrict__ level, uint32_t *__restrict__ err,
                                                  const uint32_t *__restrict__ bad, uint32_t *__restrict__ qflag) {
    if (*bad) return;  // a corrupt CSR: no expansion (uniform: every block leaves)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t sh = blockIdx.x % kShards;
    uint32_t *head = &ctl[sh * kCtlStride];
    uint32_t *done = &ctl[(2 * kShards + sh) * kCtlStride];
    uint32_t *fin = &ctl[kFinWord], *abortw = &ctl[kAbortWord];
    uint64_t *q = Q + (size_t)sh * V * 2;  // claims come from the block's own shard (2 words a slot)
    uint32_t rr = blockIdx.x / kShards;    // pushes rotate over all shards (load spreading)
    const bool monitor = blockIdx.x == 0;
    const uint64_t lt = (1ull << lane) - 1ull;
    // lane state: a claim on a queue slot, or an item u (level lu) with edges [e, e1),
    // and at most one continuation cw (level cl, edges [ce, ce1))
    // every lane starts with a claim: wave k of a shard holds its slots [64k, 64k + 64) (the heads
    // start at kInitClaims, k_lvl_zero), so the first items are polled in the first round (config 5:
    // 0.641-0.656 against 0.650-0.663 ms, profiles/r07u_lvl_ab.txt; raising a chain-walking wave's
    // s_setprio to 1 / 3 cost 8-13 us, r07v_lvl_ab.txt)
    bool has_claim = true, has_item = false;
    uint32_t slot = (blockIdx.x / kShards) * 64u + lane, u = 0, lu = 0, e = 0, e1 = 0, my_max = 0, idle = 0;
    uint32_t cw = FP_NONE, cl = 0, ce = 0, ce1 = 0;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    // two push sets, alternating by round parity (see the loop comment)
    PushSet sA, sB;
#pragma unroll
    for (uint32_t k = 0; k < kPush; ++k) sA.pend[k] = sB.pend[k] = false;
    sA.tot = sB.tot = sA.ndone = sB.ndone = 0;
    sA.ps = sB.ps = sA.pbase = sB.pbase = 0;
    // claims: needed (issued next round), reserved (read the round after), the leader, this lane's rank
    bool cneed = false, cpend = false;
    uint32_t cbase = 0, cleader = 0, crank = 0;
    // a consumed queue slot, emptied next round
    bool rs_pend = false;
    uint32_t rs_slot = 0;
#ifdef FP_LVL_TRACE
    uint32_t trL = FP_NONE;
    uint64_t trT = 0;
#endif
    // (Round 6 tried loading a join child's first edge record beside the CAS that may make it ready,
    // to save a round trip per join level on the chain: k_lvl_async 495 -> 540 us on config 5,
    // profiles/r07h_lvl_prefetch_kernel_stats.csv -- the extra loads of every join edge cost more than they saved.)
    //
    // A wave's memory operations complete in order (loads, stores and atomics on one counter), so a
    // round's wait for its edge records is also a wait for every store and atomic issued before
    // them.  A round therefore issues its records and polls first and only then the previous rounds'
    // deferred work: the queue stores of the pushes reserved one round ago (set SP), the
    // reservation of the pushes computed last round (set SQ), the done count of the items whose
    // pushes were just stored, the emptying of consumed slots, and the claims.  Every store and
    // atomic thus has a whole round to complete before a load waits behind it.  (Config 5, trace
    // build: a chain's 4-level round took 5.3 us with its side pushes and 2.3 us with them dropped,
    // profiles/r07w_*; this order brought it to 4.0-4.3 us, r07x_trace.jsonl, and the production
    // kernel 3-6 us, r07x_lvl_ab.txt.)
    // Ordering for termination: the done count of an item is issued only after the reservation of
    // its children's slots has returned (the wait on SP.pbase), so done never overtakes tail.
    auto round = [&](PushSet &SP, PushSet &SQ) -> bool {
        // a vertex with many edges left (a chain head feeding a whole fan-out layer) is expanded by
        // the whole wave, 64 edges per step (below); the others take one edge step per lane
        const bool coop = has_item && e1 - e >= kCoopEdges;
        uint64_t bm = __ballot(coop);
        bool ready[kLaneEdges], fin_item = false, part = false;
        bool jp[kHops - 1];  // a vertex passed by a jump has edges left: queue them
        QEnt jent[kHops - 1];
#pragma unroll
        for (uint32_t h = 0; h + 1 < kHops; ++h) jp[h] = false;
        QEnt pent_part{0, 0};
        uint32_t w[kLaneEdges], wl[kLaneEdges], p0[kLaneEdges], p1[kLaneEdges];
#pragma unroll
        for (uint32_t k = 0; k < kLaneEdges; ++k) ready[k] = false;
        const uint32_t ne = has_item && !coop ? min(e1 - e, kLaneEdges) : 0u;
        uint4 erv[kLaneEdges], erh[kHops - 1];
#pragma unroll
        for (uint32_t k = 0; k < kLaneEdges; ++k)
            if (k < ne) erv[k] = erec[e + k];
#pragma unroll
        for (uint32_t h = 0; h + 1 < kHops; ++h)  // the hops after edge e (k_edge_hops), same round trip
            erh[h] = ne ? erec2[(size_t)h * E + e] : make_uint4(0u, 0u, 0u, 0u);
#ifdef FP_LVL_TRACE
        const uint32_t trL0 = trL;
        const uint64_t trT0 = trT;
        unsigned long long trV = 0;
        if (trL0 != FP_NONE) trV = __hip_atomic_load(&g_lvl_trace[trL0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        trL = FP_NONE;
#endif
        // the poll of a claimed slot, behind the records
        QEnt x{kQEmpty, kQEmpty};
        // (polling the first word alone, and the second once the first is set, halves the poll
        // loads but delays every pickup by a round: config 5 +17 us, profiles/r08k_lvl_ab.txt;
        // polling only slots below the shard's tail as last read, which skips unreserved slots,
        // took 0.79-0.82 ms -- every wave reading the hot tail words each round, r08t_lvl_ab.txt)
        if (has_claim && slot < V) {
            x.lo = ag_ld64(&q[2 * (size_t)slot]);
            x.hi = ag_ld64(&q[2 * (size_t)slot + 1]);
        }
        // ---- the deferred work, behind this round's loads
        if (SP.tot) {  // reserved at the previous round's top: store the entries
            const uint32_t base = __shfl(SP.pbase, 0);
            uint64_t *pq = Q + (size_t)SP.ps * V * 2;
#pragma unroll
            for (uint32_t k = 0; k < kPush; ++k)
                if (SP.pend[k]) q_store(pq + 2 * (size_t)(base + SP.pofs[k]), SP.pent[k]);
            SP.tot = 0;
        }
        if (SP.ndone) {  // their items are done (relaxed, not waited for)
            if (lane == 0) __hip_atomic_fetch_add(done, SP.ndone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            SP.ndone = 0;
        }
        if (SQ.tot && lane == 0) SQ.pbase = atomicAdd(&ctl[(kShards + SQ.ps) * kCtlStride], SQ.tot);
        if (rs_pend) {  // the slot consumed last round: empty again (a clean finish leaves the queues empty)
            q_store(&q[2 * (size_t)rs_slot], QEnt{kQEmpty, kQEmpty});
            rs_pend = false;
        }
        if (__ballot(cpend)) {  // last round's claim reservation: the slot is polled next round
            const uint32_t b = __shfl(cbase, (int)cleader);
            if (cpend) {
                slot = b + crank;
                has_claim = true;
                cpend = false;
            }
        }
        {  // claim one queue slot per lane without work (wave-aggregated)
            const uint64_t nm = __ballot(cneed);
            if (nm) {
                cleader = (uint32_t)__builtin_ctzll(nm);
                if (lane == cleader) cbase = atomicAdd(head, (uint32_t)__popcll(nm));
                if (cneed) {
                    crank = (uint32_t)__popcll(nm & lt);
                    cpend = true;
                    cneed = false;
                }
            }
        }
        while (bm) {
            const uint32_t L = (uint32_t)__builtin_ctzll(bm);
            bm &= bm - 1;
            const uint32_t blu = __builtin_amdgcn_readlane(lu, L), be0 = __builtin_amdgcn_readlane(e, L),
                           be1 = __builtin_amdgcn_readlane(e1, L);
            for (uint32_t base = be0; base < be1; base += 64) {
                const uint32_t ee = base + lane;
                bool rdy = false;
                uint32_t ww = 0, r0 = 0, r1 = 0;
                uint64_t cur = 0;
                if (ee < be1) {
                    const uint4 er = erec[ee];
                    ww = er.x; r0 = er.y; r1 = er.z;
                    uint64_t exp = (1ull << 32) | 1ull;
                    if (er.w) cur = (uint64_t)(blu + 1u) << 32;  // the only parent: ready, no atomic
                    else
                    while (true) {
                        const uint32_t nl = max((uint32_t)(exp >> 32), blu + 1u);
                        const uint64_t nv = ((uint64_t)nl << 32) | (uint32_t)((uint32_t)exp - 1u);
                        uint64_t obs = exp;
                        if (__hip_atomic_compare_exchange_strong(&state[ww], &obs, nv, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                            cur = nv;
                            break;
                        }
                        exp = obs;
                    }
                    if ((uint32_t)cur == 0u) {
                        const uint32_t wl0 = (uint32_t)(cur >> 32);
                        if (r1 > r0) rdy = true;
                        else {  // no out-edges: final here
                            level[ww] = wl0;
                            my_max = max(my_max, wl0);
                        }
                    }
                }
                // these pushes are stored at once, after their reservation returns: the items
                // they finish are counted in a later round, behind the stores
                const uint64_t rm = __ballot(rdy);
                if (rm) {
                    const uint32_t leader = (uint32_t)__builtin_ctzll(rm);
                    uint32_t b0 = 0;
                    const uint32_t ps = (sh + ++rr) % kShards;
                    if (lane == leader) b0 = atomicAdd(&ctl[(kShards + ps) * kCtlStride], (uint32_t)__popcll(rm));
                    b0 = __shfl(b0, (int)leader);
                    if (rdy)
                        q_store(Q + ((size_t)ps * V + b0 + (uint32_t)__popcll(rm & lt)) * 2,
                                q_ent(ww, (uint32_t)(cur >> 32), r0, r1));
                }
            }
            if (lane == L) e = e1;  // the step below finishes (or continues) the item
        }
        if (has_item) {
            uint64_t cur[kLaneEdges], obs[kLaneEdges];
            bool only[kLaneEdges];
#pragma unroll
            for (uint32_t k = 0; k < kLaneEdges; ++k)
                if (k < ne) {  // the child and its edge range (the continuation's) in one record
                    const uint4 er = erv[k];
                    w[k] = er.x; p0[k] = er.y; p1[k] = er.z; only[k] = er.w != 0u;
                }
            // first attempt guesses an untouched vertex with deps and one parent (a chain link)
            const uint64_t g = (1ull << 32) | 1ull;
            const uint64_t gn = ((uint64_t)max(1u, lu + 1u) << 32);
#pragma unroll
            for (uint32_t k = 0; k < kLaneEdges; ++k) {
                if (k < ne) {
                    obs[k] = g;
                    cur[k] = only[k] ? gn  // this edge is the child's only in-edge: ready, no atomic
                                     : __hip_atomic_compare_exchange_strong(&state[w[k]], &obs[k], gn, __ATOMIC_RELAXED,
                                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           ? gn : kQEmpty;
                }
            }
#pragma unroll
            for (uint32_t k = 0; k < kLaneEdges; ++k) {
                if (k < ne) {
                    uint64_t exp = obs[k];
                    while (cur[k] == kQEmpty) {  // retry with the observed word
                        const uint32_t nl = max((uint32_t)(exp >> 32), lu + 1u);
                        const uint64_t nv = ((uint64_t)nl << 32) | (uint32_t)((uint32_t)exp - 1u);
                        uint64_t o = exp;
                        if (__hip_atomic_compare_exchange_strong(&state[w[k]], &o, nv, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                            cur[k] = nv;
                        else
                            exp = o;
                    }
                    if ((uint32_t)cur[k] == 0u) {
                        wl[k] = (uint32_t)(cur[k] >> 32);
                        if (p1[k] == p0[k]) {  // no out-edges: final here, nothing to queue
                            level[w[k]] = wl[k];
                            LVL_TR(wl[k]);
                            my_max = max(my_max, wl[k]);
                        } else if (cw == FP_NONE) {
                            cw = w[k]; cl = wl[k]; ce = p0[k]; ce1 = p1[k];
                            // the jump: w ready through its only parent (this edge) and its first
                            // dependent ready through w alone (and so on, kHops - 1 times) -- each
                            // passed vertex is final here, the lane continues at the last one, and
                            // the passed vertices' other edges are queued as partial items
                            if (k == 0 && only[0]) {
                                bool go = true;
#pragma unroll
                                for (uint32_t h = 0; h + 1 < kHops; ++h) {
                                    go = go && erh[h].w != 0u;
                                    if (go) {
                                        level[cw] = cl;
                                        LVL_TR(cl);
                                        my_max = max(my_max, cl);
                                        if (ce + 1u < ce1) {
#ifndef LVL_DROP_JP  // diagnostics only: wrong levels, times the chain walk without its side pushes
                                            jp[h] = true;
#endif
#ifdef LVL_SKIP_SIDE  // diagnostics only: side items are taken and dropped (wrong levels)
                                            jent[h] = q_ent(cw, cl | 0x80000000u, ce + 1u, ce1);
#else
                                            jent[h] = q_ent(cw, cl, ce + 1u, ce1);
#endif
                                        }
                                        cw = erh[h].x; cl = cl + 1u; ce = erh[h].y; ce1 = erh[h].z;
                                    }
                                }
                            }
                        } else {
                            ready[k] = true;
                        }
                    }
                }
            }
            e += ne;
            // a continuation with edges of u left: hand those to the queue as a partial item
            // and follow the chain now
            if (cw != FP_NONE && e < e1) {
#ifndef LVL_DROP_JP
                part = true;
#endif
#ifdef LVL_SKIP_SIDE
                pent_part = q_ent(u, lu | 0x80000000u, e, e1);
#else
                pent_part = q_ent(u, lu, e, e1);
#endif
                e = e1;
            }
            if (e >= e1) {
                if (cw != FP_NONE) {  // continue down the chain in this lane
                    u = cw; lu = cl; e = ce; e1 = ce1;
                    cw = FP_NONE;
                    level[u] = lu;
                    LVL_TR(lu);
                    my_max = max(my_max, lu);
                } else {
                    has_item = false;
                    fin_item = true;
                }
            }
        }
#ifdef LVL_SKIP_SIDE
        if (x.lo != kQEmpty && x.hi != kQEmpty && (x.lo >> 63)) {
            rs_pend = true;
            rs_slot = slot;
            has_claim = false;
            fin_item = true;
            x.lo = kQEmpty;
        }
#endif
        if (x.lo != kQEmpty && x.hi != kQEmpty) {  // a claimed item arrived
            rs_pend = true;
            rs_slot = slot;
            has_claim = false;
            has_item = true;
            u = (uint32_t)x.lo;
            lu = (uint32_t)(x.lo >> 32);
            e = (uint32_t)(x.hi >> 32);
            e1 = (uint32_t)x.hi;
            level[u] = lu;
            LVL_TR(lu);
            my_max = max(my_max, lu);
        }
        cneed = !has_claim && !has_item && !cpend;
        // this round's pushes into SP: reserved next round (as that round's SQ), stored the round
        // after; entries: [0, kLaneEdges) ready children, then the jumps' partial items, then u's part
        bool pp[kPush];
        QEnt pe[kPush];
#pragma unroll
        for (uint32_t k = 0; k < kLaneEdges; ++k) {
            pp[k] = ready[k];
            pe[k] = q_ent(w[k], wl[k], p0[k], p1[k]);
        }
#pragma unroll
        for (uint32_t h = 0; h + 1 < kHops; ++h) {
            pp[kLaneEdges + h] = jp[h];
            pe[kLaneEdges + h] = jent[h];
        }
        pp[kPush - 1] = part;
        pe[kPush - 1] = pent_part;
        uint64_t rm[kPush];
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t k = 0; k < kPush; ++k) {
            rm[k] = __ballot(pp[k]);
            tot += (uint32_t)__popcll(rm[k]);
        }
        SP.tot = tot;
        if (tot) {
            SP.ps = (sh + ++rr) % kShards;
            uint32_t run = 0;
#pragma unroll
            for (uint32_t k = 0; k < kPush; ++k) {
                SP.pend[k] = pp[k];
                SP.pofs[k] = run + (uint32_t)__popcll(rm[k] & lt);
                SP.pent[k] = pe[k];
                run += (uint32_t)__popcll(rm[k]);
            }
        }
        SP.ndone = (uint32_t)__popcll(__ballot(fin_item));
#ifdef FP_LVL_TRACE
        if (trL0 != FP_NONE && trV > trT0) atomicMin(&g_lvl_trace[trL0], (unsigned long long)trT0);
#endif
        // busy while anything is in hand or deferred
        if (__ballot(has_item || rs_pend) || SP.tot || SP.ndone || SQ.tot || SQ.ndone) {
            idle = 0;
            return false;
        }
        // idle round: every lane holds a claim (or a reservation) on an empty (or past-the-end)
        // slot, and nothing is deferred
        uint32_t stop = 0;
        if (lane == 0) {
            if (monitor) {
                uint32_t d = 0, t = 0;
                for (uint32_t k = 0; k < kShards; ++k) d += ag_rmw_rd(&ctl[(2 * kShards + k) * kCtlStride]);
                for (uint32_t k = 0; k < kShards; ++k) t += ag_rmw_rd(&ctl[(kShards + k) * kCtlStride]);
                if (d == t) {
                    __hip_atomic_store(fin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (qflag) __hip_atomic_store(qflag, kQClean, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    stop = 1;
                }
            }
            if (ag_ld32(fin) || ag_ld32(abortw)) stop = 1;
            if (!stop && __builtin_amdgcn_s_memrealtime() - t_start > 100ull * 1000 * 1000 * 60) {  // 60 s guard
                __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicMax(err, (uint32_t)(-FP_EDEVICE));
                stop = 1;
            }
        }
        if (__shfl(stop, 0)) return true;
        ++idle;
        if (idle < LVL_IDLE_SPIN) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(LVL_SLEEP_LONG);
        return false;
    };
    // rounds alternate the sets: a round stores SP (reserved in the round before), reserves SQ
    // (computed in the round before) and computes its own pushes into SP
    while (true) {
        if (round(sA, sB)) break;
        if (round(sB, sA)) break;
    }
    for (int o = 32; o > 0; o >>= 1) my_max = max(my_max, (uint32_t)__shfl_xor((int)my_max, o));
    // most waves never saw the top level: a load first keeps them off the one contended word (config 5:
    // k_lvl_async -5 to -10 us, profiles/r07n_lvl_ab.txt)
    if (lane == 0 && my_max && my_max > ag_ld32(&ctl[kMaxLevelWord])) atomicMax(&ctl[kMaxLevelWord], my_max);
#ifdef FP_LVL_TRACE
    if (lane == 0) {
        atomicMin(&g_lvl_trace[4094], t_start);
        atomicMax(&g_lvl_trace[4095], __builtin_amdgcn_s_memrealtime());
    }
#endif
}

// level -> sort keys; vertices never finished (cycle members and everything behind
// them) are NONE and take the cycle key, which sorts after every level: max(largest level, 1)
// + 1, from the largest level the async kernel recorded (ctl maxlvl), computed here on the
// device and left in *ck for the sort; counts the NONE vertices.
__global__ void k_lvl_async_final(uint32_t V, const uint32_t *__restrict__ ctl, const uint32_t *__restrict__ level,
                                  uint32_t *__restrict__ keys, uint32_t *__restrict__ vals, uint32_t *__restrict__ ncyc,
                                  uint32_t *__restrict__ ck,
                                  const uint32_t *__restrict__ bad, uint32_t *__restrict__ ncyc_out) {
    if (*bad) return;
    const uint32_t maxl = ctl[kMaxLevelWord];
    const uint32_t cyc_key = (maxl > 1 ? maxl : 1u) + 1u;
    if (blockIdx.x == 0 && threadIdx.x == 0) *ck = cyc_key;
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool cyc = v < V && level[v] == FP_NONE;
    if (v < V) {
        keys[v] = cyc ? cyc_key : level[v];
        if (vals) vals[v] = (uint32_t)v;  // the radix fallback's values (null for the counting sort)
    }
    const uint64_t m = __ballot(cyc);
    if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) {
        atomicAdd(ncyc, (uint32_t)__popcll(m));
        if (ncyc_out) atomicAdd(ncyc_out, (uint32_t)__popcll(m));
    }
}

// ---- stable counting sort of the level keys (the start order) ----------------------------
// LSD over CS_BITS-bit digits: pass p orders by bits [p * CS_BITS, (p + 1) * CS_BITS) of the key,
// stably, so after the last pass the vertices are in (level, index) order.  Three small launches
// per pass instead of rocprim's ~21 radix launches (launch-bound at config 5's 1M keys: 0.16 ms):
//   k_cs_hist    per tile of CS_TILE keys: a histogram of the pass's digit in LDS -> hist[tile][bin]
//   k_cs_scan    one workgroup: hist[tile][bin] <- bin base + keys of the bin in earlier tiles
//   k_cs_scatter per tile: per-wave counts of each wave's contiguous slice, then each wave walks
//                its slice in order, 64 keys at a time, ranking equal digits by a ballot match
//                mask (the same stable scheme as fp_place.hip's per-scenario sort)
// The key range is a DEVICE value (*ck: the cycle key, the largest key): a pass beyond the digits
// it needs returns at once, the last needed pass writes the vertex order to `order`, and earlier
// passes ping-pong (key, vertex) pairs through two scratch pairs.  The host enqueues the passes V
// could need (ceil(bits(V + 1) / CS_BITS)) and reads nothing back: config 5's 509 levels take one
// pass and the others return at once.
// tiles of 16384 keys: config 5's 1M keys are 62 workgroups; 4096 / 8192 / 12288-key tiles ran
// 0.693-0.699 / 0.653-0.656 / 0.651-0.660 ms against 0.653-0.656 (profiles/r07r_lvl_ab.txt); with the
// fused late passes 8192 (128 register tiles) / 24576 / 32768 keys 0.634-0.635 / 0.630 / 0.633-0.635
// against 0.624 ms (profiles/r09m_lvl_ab.txt)
#ifndef CS_TILE_KEYS
#define CS_TILE_KEYS 16384
#endif
#ifndef CS_REG_TILES
#define CS_REG_TILES 64
#endif
constexpr uint32_t CS_TILE = CS_TILE_KEYS, CS_BITS = 10, CS_BINS = 1u << CS_BITS, CS_WAVES = 16, CS_MAX_TILES = 1024;
constexpr uint32_t kCsPassesMax = (32 + CS_BITS - 1) / CS_BITS;  // passes a 32-bit key can need

struct CsPass {
    uint32_t sh, nb, nbits;  // digit shift, bins (digits < nb), bits the match masks test
    bool active, last;
};
__device__ __forceinline__ CsPass cs_pass_k(uint32_t p, uint32_t kmax) {
    const uint32_t bits = kmax ? 32u - (uint32_t)__builtin_clz(kmax) : 1u;
    const uint32_t need = (bits + CS_BITS - 1u) / CS_BITS;
    CsPass c;
    c.sh = p * CS_BITS;
    c.active = p < need;
    c.last = p + 1u == need;
    c.nb = c.last ? (kmax >> c.sh) + 1u : CS_BINS;
    c.nbits = c.nb > 1u ? 32u - (uint32_t)__builtin_clz(c.nb - 1u) : 0u;
    return c;
}
__device__ __forceinline__ CsPass cs_pass(uint32_t p, const uint32_t *ck) { return cs_pass_k(p, *ck); }
// the error word and the key range in one round trip (a pass that is not needed returns after it)
__device__ __forceinline__ bool cs_start(const uint32_t *bad, const uint32_t *ck, uint32_t &kmax) {
    const uint32_t b = *bad;
    kmax = *ck;
    return b == 0u;
}
// The asynchronous levelizer sorts its levels in place of keys (LvlMap): pass 0 reads level[] and
// sorts a CYCLE vertex (FP_NONE) under the cycle key, max(largest level, 1) + 1, which k_cs_hist
// derives from the schedule's largest level and publishes for the later kernels (no key array
// and no separate key kernel).
struct LvlMap {
    const uint32_t *maxl;  // null: the keys are plain keys; else the async schedule's largest level
    uint32_t *ncyc, *ncyc_out;  // cycle counts (k_cs_hist, pass 0)
};
__device__ __forceinline__ uint32_t cs_key(uint32_t k, uint32_t ckey) { return k == FP_NONE ? ckey : k; }
__device__ __forceinline__ uint32_t cs_digit(uint32_t key, const CsPass &c) {
    return min(c.last ? key >> c.sh : (key >> c.sh) & (CS_BINS - 1u), c.nb - 1u);
}

__device__ __forceinline__ uint64_t cs_match(uint32_t v, bool valid, uint32_t nbits) {
    uint64_t m = __builtin_amdgcn_ballot_w64(valid);
    for (uint32_t i = 0; i < nbits; ++i) {
        const bool bit = (v >> i) & 1u;
        const uint64_t bb = __builtin_amdgcn_ballot_w64(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}
// the tile's histogram of the pass digit (LDS) -> its row of hist (keys already loaded: kv[j] is
// key t0 + threadIdx.x + 1024 j); map: levels as keys, counting the cycle vertices
template <uint32_t PER>
__device__ __forceinline__ void cs_hist_tile(const uint32_t (&kv)[PER], size_t t0, uint32_t V, const CsPass &c,
                                             bool map, uint32_t ckey, uint32_t *__restrict__ row, uint32_t &ncy) {
    __shared__ uint32_t h[CS_BINS];
    for (uint32_t b = threadIdx.x; b < c.nb; b += blockDim.x) h[b] = 0;
    __syncthreads();
    const uint32_t wbase = threadIdx.x & ~63u;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        if (t0 + wbase + j * 1024u >= V) break;  // wave-uniform
        const bool valid = t0 + threadIdx.x + j * 1024u < V;
        uint32_t k = kv[j];
        if (map) {
            ncy += valid && k == FP_NONE ? 1u : 0u;
            k = cs_key(k, ckey);
        }
        const uint32_t d = valid ? cs_digit(k, c) : 0u;
        // (counting equal digits once per wave by their match masks instead: hist 12.1 -> 17.6 us,
        // scatter 16.8 -> 25.3 us on config 5, profiles/r08a_lvl_ab.txt -- the ballots cost more than
        // the LDS conflicts they avoid)
        if (valid) atomicAdd(&h[d], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < c.nb; b += blockDim.x) row[b] = h[b];
}

// one workgroup of CS_BINS threads: hist[tile][bin] <- bin base + keys of the bin in earlier tiles
__device__ __forceinline__ void cs_scan_bins(uint32_t *__restrict__ hist, uint32_t ntiles, uint32_t nb) {
    __shared__ uint32_t tot[CS_BINS / 64];  // the waves' sums
    const uint32_t b = threadIdx.x;  // one bin per thread (nb <= CS_BINS = blockDim)
    constexpr uint32_t REG_TILES = CS_REG_TILES;  // up to 1M keys: the bin's counts stay in registers
    uint32_t x[REG_TILES];
    uint32_t run = 0;
    const bool in_regs = ntiles <= REG_TILES;
    if (b < nb) {
        if (in_regs) {  // every load in flight at once, one round trip; the prefix in registers
#pragma unroll
            for (uint32_t t = 0; t < REG_TILES; ++t) x[t] = t < ntiles ? hist[(size_t)t * nb + b] : 0u;
#pragma unroll
            for (uint32_t t = 0; t < REG_TILES; ++t) {
                const uint32_t y = x[t];
                x[t] = run;
                run += y;
            }
        } else {
            for (uint32_t t0 = 0; t0 < ntiles; t0 += 8) {  // 8 independent loads in flight
                uint32_t y[8];
#pragma unroll
                for (uint32_t j = 0; j < 8; ++j) y[j] = t0 + j < ntiles ? hist[(size_t)(t0 + j) * nb + b] : 0u;
#pragma unroll
                for (uint32_t j = 0; j < 8; ++j)
                    if (t0 + j < ntiles) {
                        hist[(size_t)(t0 + j) * nb + b] = run;
                        run += y[j];
                    }
            }
        }
    }
    // exclusive scan of the bin totals: within each wave by shuffles, then the earlier waves' sums
    // (one barrier; the LDS Hillis-Steele scan took twenty)
    const uint32_t lane = b & 63, wv = b >> 6;
    uint32_t inc = b < nb ? run : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
        if ((int)lane >= o) inc += y;
    }
    if (lane == 63) tot[wv] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t q = 0; q < wv; ++q) pre += tot[q];
    const uint32_t base = pre + inc - (b < nb ? run : 0u);
    if (b < nb) {
        if (in_regs) {
#pragma unroll
            for (uint32_t t = 0; t < REG_TILES; ++t)
                if (t < ntiles) hist[(size_t)t * nb + b] = x[t] + base;
        } else {
            for (uint32_t t = 0; t < ntiles; ++t) hist[(size_t)t * nb + b] += base;
        }
    }
}

// a wave's slice of the tile in (key, vertex) order of the pass digit: per-wave counts, the wave
// offsets from the tile's row of the scanned hist, then ranks by ballot match masks (kv already
// mapped by the caller when map; kv[j], xv[j] = key / vertex s0 + 64 j + lane)
template <uint32_t PER>
__device__ __forceinline__ void cs_scatter_slice(const uint32_t (&kv)[PER], const uint32_t (&xv)[PER], size_t s0,
                                                 uint32_t V, const CsPass &c, const uint32_t *__restrict__ offrow,
                                                 uint32_t *__restrict__ order, uint32_t *__restrict__ kout,
                                                 uint32_t *__restrict__ vout) {
    __shared__ uint32_t wh[CS_WAVES][CS_BINS];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, nb = c.nb;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t i = t; i < CS_WAVES * CS_BINS; i += blockDim.x) (&wh[0][0])[i] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        if (s0 + j * 64u >= V) break;  // wave-uniform
        if (s0 + j * 64u + lane < V) atomicAdd(&wh[w][cs_digit(kv[j], c)], 1u);
    }
    __syncthreads();
    for (uint32_t b = t; b < nb; b += blockDim.x) {  // per bin: wave offsets in wave order
        uint32_t run = offrow[b];
        for (uint32_t ww = 0; ww < CS_WAVES; ++ww) {
            const uint32_t x = wh[ww][b];
            wh[ww][b] = run;
            run += x;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        if (s0 + j * 64u >= V) break;  // wave-uniform
        const bool valid = s0 + j * 64u + lane < V;
        const uint32_t key = kv[j];
        const uint32_t k = valid ? cs_digit(key, c) : 0u;
        const uint32_t x = xv[j];
        const uint64_t m = cs_match(k, valid, c.nbits);
        const uint32_t o = wh[w][k];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every lane's read before the update
        if (valid) {
            if ((m & lt) == 0) wh[w][k] = o + (uint32_t)__popcll(m);
            const uint32_t q = o + (uint32_t)__popcll(m & lt);
            if (c.last) {
                order[q] = x;
            } else {
                kout[q] = key;
                vout[q] = x;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

constexpr uint32_t CS_HPER = CS_TILE / 1024u;               // keys per thread in a tile's histogram
constexpr uint32_t CS_SLICE = CS_TILE / CS_WAVES, CS_SPER = CS_SLICE / 64u;  // per wave / lane in the scatter

__global__ __launch_bounds__(1024) void k_cs_hist(const uint32_t *__restrict__ keys, uint32_t V, uint32_t p,
                                                  uint32_t *__restrict__ ck, const uint32_t *__restrict__ bad,
                                                  uint32_t *__restrict__ hist, LvlMap lm, uint32_t *__restrict__ bar) {
    const bool map = lm.maxl && p == 0;
    // the tile's keys are loaded with the control words, all in one round trip (a load per
    // iteration behind the LDS atomics cost a round trip each: 15.5 us for config 5's 1M keys)
    const size_t t0 = (size_t)blockIdx.x * CS_TILE;
    uint32_t kv[CS_HPER];
    auto load = [&]() {
#pragma unroll
        for (uint32_t j = 0; j < CS_HPER; ++j) {
            const size_t i = t0 + threadIdx.x + j * 1024u;
            kv[j] = i < V ? keys[i] : 0u;
        }
    };
    if (p == 0) load();  // pass 0 always runs; a later pass may not be needed (loaded below)
    const uint32_t badv = *bad, maxl = map ? *lm.maxl : 0u, ckv = map ? 0u : *ck;
    if (badv) return;
    uint32_t ckey = 0;
    if (map) {
        ckey = (maxl > 1 ? maxl : 1u) + 1u;
        if (blockIdx.x == 0 && threadIdx.x == 0) *ck = ckey;  // the later kernels read it
    }
    // pass 0 clears the barrier words of the later passes' single-launch kernel (k_cs_pass_late)
    if (p == 0 && bar && blockIdx.x == 0 && threadIdx.x < 2 * kCsPassesMax) bar[threadIdx.x] = 0u;
    const CsPass c = cs_pass_k(p, map ? ckey : ckv);
    if (!c.active) return;
    if (p != 0) load();
    uint32_t ncy = 0;
    cs_hist_tile(kv, t0, V, c, map, ckey, hist + (size_t)blockIdx.x * c.nb, ncy);
    if (map) {  // the cycle vertices: one atomic per wave that has any
        for (int o = 32; o > 0; o >>= 1) ncy += (uint32_t)__shfl_xor((int)ncy, o);
        if ((threadIdx.x & 63) == 0 && ncy) {
            atomicAdd(lm.ncyc, ncy);
            if (lm.ncyc_out) atomicAdd(lm.ncyc_out, ncy);
        }
    }
}

__global__ void k_cs_scan(uint32_t *__restrict__ hist, uint32_t ntiles, uint32_t p, const uint32_t *__restrict__ ck,
                          const uint32_t *__restrict__ bad) {
    uint32_t kmax;
    if (!cs_start(bad, ck, kmax)) return;
    const CsPass c = cs_pass_k(p, kmax);
    if (!c.active) return;
    cs_scan_bins(hist, ntiles, c.nb);
}

// pass p: (keys, vals) -> (kout, vout), or the vertices alone -> order on the last pass.
// vals null: the vertex is the key's index (pass 0).
__global__ __launch_bounds__(1024) void k_cs_scatter(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                     uint32_t V, uint32_t p, const uint32_t *__restrict__ ck,
                                                     const uint32_t *__restrict__ bad, const uint32_t *__restrict__ off,
                                                     uint32_t *__restrict__ order, uint32_t *__restrict__ kout,
                                                     uint32_t *__restrict__ vout, bool map) {
    // the wave's slice of keys (and vertices) is loaded once, with the control words, and kept in
    // registers for both walks (a load per iteration cost a round trip each: 23.4 us for config 5)
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t s0 = (size_t)blockIdx.x * CS_TILE + (size_t)w * CS_SLICE;
    uint32_t kv[CS_SPER], xv[CS_SPER];
    auto load = [&]() {
#pragma unroll
        for (uint32_t j = 0; j < CS_SPER; ++j) {
            const size_t v = s0 + j * 64u + lane;
            kv[j] = v < V ? keys[v] : 0u;
            xv[j] = v < V ? (vals ? vals[v] : (uint32_t)v) : 0u;
        }
    };
    if (p == 0) load();  // pass 0 always runs; a later pass may not be needed (loaded below)
    uint32_t kmax;
    if (!cs_start(bad, ck, kmax)) return;
    map = map && p == 0;  // levels as keys (LvlMap): *ck is the cycle key, written by k_cs_hist
    const CsPass c = cs_pass_k(p, kmax);
    if (!c.active) return;
    if (p != 0) load();
    if (map) {
#pragma unroll
        for (uint32_t j = 0; j < CS_SPER; ++j) kv[j] = cs_key(kv[j], kmax);
    }
    cs_scatter_slice(kv, xv, s0, V, c, off + (size_t)blockIdx.x * c.nb, order, kout, vout);
}

// A pass after the first in ONE launch when its tiles fit one workgroup per CU (ntiles <=
// CS_FUSED_TILES): the histogram, the scan (workgroup 0) and the scatter meet at two grid barriers.
// (The first pass, which always runs, is faster as three launches: 39.6 us fused against 12.8 + 7.0 +
// 17.0 us on config 5, profiles/r08g_lvl_ab.txt -- the other workgroups wait through the scan.)
// A pass the keys do not need returns after one round trip: config 5's second pass (509 levels, but
// V = 1M could need 20 bits) cost three launches that return at once, 16 us.  The barriers give up
// after 10 s (FP_EDEVICE) so that a grid that is not all resident cannot hang the device.
constexpr uint32_t CS_FUSED_TILES = 64;
__device__ __forceinline__ bool cs_grid_sync(uint32_t *cnt, uint32_t target, uint32_t *err) {
    __shared__ uint32_t ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();  // this workgroup's writes before its arrival
        atomicAdd(cnt, 1u);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t good = 1;
        while (ag_ld32(cnt) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100ull * 1000 * 1000 * 10) {
                atomicMax(err, (uint32_t)(-FP_EDEVICE));
                good = 0;
                break;
            }
        }
        __threadfence();  // the others' writes after their arrival
        ok = good;
    }
    __syncthreads();
    return ok != 0u;
}
__global__ __launch_bounds__(1024) void k_cs_pass_late(const uint32_t *__restrict__ keys,
                                                       const uint32_t *__restrict__ vals, uint32_t V, uint32_t p,
                                                       const uint32_t *__restrict__ ck, const uint32_t *__restrict__ bad,
                                                       uint32_t *__restrict__ hist, uint32_t ntiles,
                                                       uint32_t *__restrict__ order, uint32_t *__restrict__ kout,
                                                       uint32_t *__restrict__ vout, uint32_t *__restrict__ bar,
                                                       uint32_t *__restrict__ err) {
    uint32_t kmax;
    if (!cs_start(bad, ck, kmax)) return;
    const CsPass c = cs_pass_k(p, kmax);
    if (!c.active) return;
    {
        const size_t t0 = (size_t)blockIdx.x * CS_TILE;
        uint32_t kv[CS_HPER], ncy = 0;
#pragma unroll
        for (uint32_t j = 0; j < CS_HPER; ++j) {
            const size_t i = t0 + threadIdx.x + j * 1024u;
            kv[j] = i < V ? keys[i] : 0u;
        }
        cs_hist_tile(kv, t0, V, c, false, 0u, hist + (size_t)blockIdx.x * c.nb, ncy);
    }
    if (!cs_grid_sync(&bar[2 * p], gridDim.x, err)) return;
    if (blockIdx.x == 0) cs_scan_bins(hist, ntiles, c.nb);
    if (!cs_grid_sync(&bar[2 * p + 1], gridDim.x, err)) return;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t s0 = (size_t)blockIdx.x * CS_TILE + (size_t)w * CS_SLICE;
    uint32_t kv[CS_SPER], xv[CS_SPER];
#pragma unroll
    for (uint32_t j = 0; j < CS_SPER; ++j) {
        const size_t v = s0 + j * 64u + lane;
        kv[j] = v < V ? keys[v] : 0u;
        xv[j] = v < V ? vals[v] : 0u;
    }
    cs_scatter_slice(kv, xv, s0, V, c, hist + (size_t)blockIdx.x * c.nb, order, kout, vout);
}

// ---- small graphs: the whole levelization in one workgroup ---------------------------------
// A graph of at most LS_V vertices and LS_E edges (a fleet.kdl stage: config 1) is levelized by
// ONE launch: CSR check, in-degrees, level-synchronous Kahn and the stable (level, index) start
// order, all in LDS (fps::ls_levels, fp_small.h).  The general path's ~25 launches and memsets
// cost ~100 us of submission for a 3-service stage; this one costs one.  FP_OPT_LEVEL_SMALL = 0
// keeps the general path.
using fps::LS_E;
using fps::LS_V;
__host__ __device__ inline size_t ls_lds_bytes(uint32_t V) { return fps::ls_words(V) * 4; }

__global__ __launch_bounds__(1024) void k_lvl_small(const uint32_t *__restrict__ row_ptr,
                                                    const uint32_t *__restrict__ col,
                                                    const uint8_t *__restrict__ hd, uint32_t V, uint32_t E,
                                                    uint32_t *__restrict__ level, uint32_t *__restrict__ order,
                                                    uint32_t *__restrict__ ncyc_out, uint32_t *__restrict__ err) {
    extern __shared__ uint32_t lsm[];
    const uint32_t nc = fps::ls_levels(row_ptr, col, hd, V, E, lsm, level, order);
    if (nc == FP_NONE) {
        if (threadIdx.x == 0) atomicMax(err, (uint32_t)(-FP_ECORRUPT));
        return;
    }
    if (threadIdx.x == 0 && ncyc_out) *ncyc_out = nc;
}

inline unsigned blocks_for(size_t n, unsigned b) {
    size_t g = (n + b - 1) / b;
    return (unsigned)(g ? g : 1);
}

}  // namespace

int fp_dev_legacy_order_impl(fp_ctx *c, const fp_graph *g, uint32_t *perm) {
    const uint32_t V = g->n_vertices;
    if (V == 0) return FP_OK;
    if (!g->has_deps || !perm) return FP_EINVAL;
    hipStream_t st = c->stream;
    if (V <= 1024 && fp_opt(c, FP_OPT_LEVEL_SMALL, 1) != 0) {  // one launch (FP_OPT_LEVEL_SMALL = 0: three)
        hipEvent_t ev;
        fp_prof_begin(c, FP_K_LEVEL, &ev);
        k_part_small<<<1, 1024, 0, st>>>(g->has_deps, V, perm);
        FP_HIP(hipGetLastError());
        fp_prof_end(c, FP_K_LEVEL, ev);
        return FP_OK;
    }
    const uint32_t nb = (uint32_t)((V + kSpan - 1) / kSpan);
    int rc = fp_ws_reserve(c, (size_t)(nb + 1) * 8 + 1024);
    if (rc) return rc;
    fp_ws_reset(c);
    uint32_t *blk_zero = (uint32_t *)fp_ws_take(c, (size_t)nb * 4 + 4);
    uint32_t *blk_off = (uint32_t *)fp_ws_take(c, (size_t)(nb + 1) * 4);
    if (!blk_zero || !blk_off) return FP_ENOMEM;
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_LEVEL, &ev);
    k_part_count<<<nb, kBlock, 0, st>>>(g->has_deps, V, blk_zero);
    FP_HIP(hipGetLastError());
    k_part_scan<<<1, 1024, 0, st>>>(blk_zero, nb, blk_off);
    FP_HIP(hipGetLastError());
    k_part_scatter<<<nb, kBlock, 0, st>>>(g->has_deps, V, blk_off, nb, perm);
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_LEVEL, ev);
    return FP_OK;
}

// order = stable sort of 0..V-1 by keys[] (keys <= *ck, a device value): the LSD counting sort
// above when its tiles cover V, else (or with FP_OPT_LEVEL_SORT = 0) rocprim's radix sort over all
// 32 key bits (vals = the identity, k_lvl_*final).  No read-back either way.  Scratch: two
// (key, vertex) pairs, kb[0]/vb[0] and kb[1]/vb[1].
#ifndef CS_FUSE_LATE
#define CS_FUSE_LATE 1  // passes after the first in one launch (k_cs_pass_late) when the tiles allow
#endif
static int level_sort(hipStream_t st, bool counting, uint32_t *keys, uint32_t *const kb[2], uint32_t *const vb[2],
                      uint32_t *order, uint32_t V, uint32_t *ck, const uint32_t *bad, void *tmp,
                      size_t sort_tmp, uint32_t *cs_hist, uint32_t *err,
                      LvlMap lm = LvlMap{nullptr, nullptr, nullptr}) {
    const uint32_t ntiles = (uint32_t)(((size_t)V + CS_TILE - 1) / CS_TILE);
    if (counting && ntiles <= CS_MAX_TILES) {
        // the largest key either schedule can produce: the async cycle key is max(level, 1) + 1 <=
        // V + 1; the level-synchronous one is iters + 2 <= (V + 1) + 2: V + 3
        const uint32_t passes = (fp_bitwidth((uint64_t)V + 3) + CS_BITS - 1) / CS_BITS;
        uint32_t *bar = cs_hist + (size_t)CS_MAX_TILES * CS_BINS;  // the late passes' barrier words
        for (uint32_t p = 0; p < passes; ++p) {
            const uint32_t *ik = p ? kb[(p - 1) & 1] : keys;
            const uint32_t *iv = p ? vb[(p - 1) & 1] : nullptr;
            if (CS_FUSE_LATE && p && ntiles <= CS_FUSED_TILES) {
                k_cs_pass_late<<<ntiles, 1024, 0, st>>>(ik, iv, V, p, ck, bad, cs_hist, ntiles, order, kb[p & 1],
                                                        vb[p & 1], bar, err);
                FP_HIP(hipGetLastError());
                continue;
            }
            k_cs_hist<<<ntiles, 1024, 0, st>>>(ik, V, p, ck, bad, cs_hist, lm, bar);
            FP_HIP(hipGetLastError());
            k_cs_scan<<<1, CS_BINS, 0, st>>>(cs_hist, ntiles, p, ck, bad);
            FP_HIP(hipGetLastError());
            k_cs_scatter<<<ntiles, 1024, 0, st>>>(ik, iv, V, p, ck, bad, cs_hist, order, kb[p & 1], vb[p & 1],
                                                  lm.maxl != nullptr);
            FP_HIP(hipGetLastError());
        }
        return FP_OK;
    }
    FP_HIP(rocprim::radix_sort_pairs(tmp, sort_tmp, keys, kb[0], vb[1], order, (size_t)V, 0, 32, st));
    return FP_OK;
}

int fp_dev_levelize_impl(fp_ctx *c, const fp_graph *g, uint32_t *level, uint32_t *order,
                         uint32_t *n_cycle_dev) {
    const uint32_t V = g->n_vertices, E = g->n_edges;
    if (V == 0) {
        if (E) return FP_ECORRUPT;
        if (n_cycle_dev) FP_HIP(hipMemsetAsync(n_cycle_dev, 0, 4, c->stream));
        return FP_OK;
    }
    if (!g->has_deps || !g->row_ptr || (E && !g->col) || !level || !order) return FP_EINVAL;
    hipStream_t st = c->stream;

    size_t sort_tmp = 0;
    FP_HIP(rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                     (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)V, 0, 32, st));
    // cnt[L] = frontier size of level L (one counter per possible level: <= V + 1)
    const size_t ncnt = (size_t)V + 2;
    // FP_OPT_LEVELIZE_SYNC = 1: the level-synchronous schedule (one launch per level); only the
    // asynchronous one takes the vertex states, queues and edge / hop records, and only the
    // counting sort (FP_OPT_LEVEL_SORT, on by default) its histograms
    const bool level_sync = fp_opt(c, FP_OPT_LEVELIZE_SYNC, 0) != 0;
    const bool counting = fp_opt(c, FP_OPT_LEVEL_SORT, 1) != 0;
    if (V <= LS_V && E <= LS_E && !level_sync && fp_opt(c, FP_OPT_LEVEL_SMALL, 1) != 0) {  // one launch
        hipEvent_t ev;
        fp_prof_begin(c, FP_K_LEVEL, &ev);
        k_lvl_small<<<1, 1024, ls_lds_bytes(V), st>>>(g->row_ptr, g->col, g->has_deps, V, E, level, order, n_cycle_dev,
                                                      c->d_err);
        FP_HIP(hipGetLastError());
        fp_prof_end(c, FP_K_LEVEL, ev);
        return FP_OK;
    }
    // the binned in-degree count (k_indeg_bin / k_indeg_hist) when the buckets fit its tables
    uint32_t bin_shift = kBinMinShift;
    while (bin_shift < kBinMaxShift && ((V + (1u << bin_shift) - 1) >> bin_shift) > kBinMaxB) ++bin_shift;
    const uint32_t bin_b = (uint32_t)(((size_t)V + (1u << bin_shift) - 1) >> bin_shift);
    const uint32_t bin_nwg = (uint32_t)(((size_t)E + kBinSlice - 1) / kBinSlice);
    const bool binned_indeg = !level_sync && E && bin_b <= kBinMaxB && fp_opt(c, FP_OPT_INDEG_BIN, 1) != 0;
    const size_t bin_ws = binned_indeg ? (size_t)E * 4 + (size_t)(bin_b + 1) * bin_nwg * 4 + (size_t)V * 16 + 768 : 0;
    const size_t async_ws = level_sync ? 0 : (size_t)V * 8 + (size_t)E * 16 * kHops + kCtlWords * 4 + bin_ws;
    const size_t cs_ws = counting ? (size_t)CS_MAX_TILES * CS_BINS * 4 + 256 : 0;  // + the barrier words
    int rc = fp_ws_reserve(c, (size_t)V * 4 * 6 + ncnt * 4 + sort_tmp + async_ws + cs_ws + 23 * 256);
    if (rc) return rc;
    fp_ws_reset(c);
    uint32_t *indeg = (uint32_t *)fp_ws_take(c, (size_t)V * 4);
    uint32_t *fa = (uint32_t *)fp_ws_take(c, (size_t)V * 4);
    uint32_t *fb = (uint32_t *)fp_ws_take(c, (size_t)V * 4);
    uint32_t *keys = (uint32_t *)fp_ws_take(c, (size_t)V * 4);
    uint32_t *keys_out = (uint32_t *)fp_ws_take(c, (size_t)V * 4);
    uint32_t *vals = (uint32_t *)fp_ws_take(c, (size_t)V * 4);
    uint32_t *cnt = (uint32_t *)fp_ws_take(c, ncnt * 4);
    uint32_t *ncyc = (uint32_t *)fp_ws_take(c, 64);
    void *tmp = fp_ws_take(c, sort_tmp + 16);
    uint32_t *cs_hist = counting ? (uint32_t *)fp_ws_take(c, cs_ws) : nullptr;
    if (!indeg || !fa || !fb || !keys || !keys_out || !vals || !cnt || !ncyc || !tmp || (counting && !cs_hist))
        return FP_ENOMEM;

    // ncyc[0]: cycle vertices; ncyc[4]: this call's corrupt-CSR flag (k_check_csr / k_indeg; every
    // later kernel reads it and does nothing); ncyc[8]: the cycle key = the largest sort key
    uint32_t *bad = ncyc + 4, *ck = ncyc + 8;
    uint32_t *const kb[2] = {keys_out, fa}, *const vb[2] = {fb, vals};  // sort scratch; vals = identity
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_LEVEL, &ev);
    if (!level_sync) {
        if ((uint64_t)V + 65536ull * 64 >= 0xFFFFFFFFull) return FP_EOVERFLOW;  // queue heads stay below 2^32
        uint64_t *state = (uint64_t *)fp_ws_take(c, (size_t)V * 8);
        uint32_t *actl = (uint32_t *)fp_ws_take(c, kCtlWords * 4);
        uint4 *erec = E ? (uint4 *)fp_ws_take(c, (size_t)E * 16) : nullptr;
        uint4 *erec2 = E ? (uint4 *)fp_ws_take(c, (size_t)E * 16 * (kHops - 1)) : nullptr;
        if (!state || !actl || (E && (!erec || !erec2))) return FP_ENOMEM;
        // the queues: the context's own buffer, emptied by the device only when dirty (kQClean)
        const size_t qbytes = (size_t)V * 16 * kShards;  // 16-B entries (k_lvl_async)
        if (qbytes + 256 > c->lvl_q_cap) {
            FP_HIP(hipStreamSynchronize(st));
            if (c->lvl_q) (void)hipFree(c->lvl_q);
            c->lvl_q = nullptr;
            c->lvl_q_cap = 0;
            const size_t cap = (qbytes + qbytes / 4 + 4096 + 255) & ~(size_t)255;
            FP_HIP(hipMalloc(&c->lvl_q, cap));
            c->lvl_q_cap = cap;
            FP_HIP(hipMemsetAsync((char *)c->lvl_q + cap - 256, 0, 256, st));  // flag: dirty
        }
        uint64_t *Q = (uint64_t *)c->lvl_q;
        uint32_t *qflag = (uint32_t *)((char *)c->lvl_q + c->lvl_q_cap - 256);
        const unsigned zg = blocks_for((c->lvl_q_cap - 256) / 16, 256) < 8192 ? blocks_for((c->lvl_q_cap - 256) / 16, 256) : 8192;
        // "clean" covers the WHOLE buffer: a dirty buffer is refilled to its capacity, not to this
        // call's queue size, so a later call with a larger graph (a larger queue in the same
        // buffer) never reads slots an earlier, smaller call left unfilled
        const size_t qfill = c->lvl_q_cap - 256;
        // (the binned count stores every in-degree itself: no zeroing)
        k_lvl_zero<<<zg, 256, 0, st>>>(binned_indeg ? 0u : V, indeg, ncyc, actl, n_cycle_dev, (uint4 *)Q, qfill / 16,
                                       qflag);
        FP_HIP(hipGetLastError());
        const size_t nmax = V + 1 > E ? (size_t)V + 1 : E;
        uint4 *vrec = nullptr;  // per-vertex edge-record halves (binned path)
        if (binned_indeg) {
            uint32_t *binned = (uint32_t *)fp_ws_take(c, (size_t)E * 4);
            uint32_t *offt = (uint32_t *)fp_ws_take(c, (size_t)(bin_b + 1) * bin_nwg * 4);
            vrec = (uint4 *)fp_ws_take(c, (size_t)V * 16);
            if (!binned || !offt || !vrec) return FP_ENOMEM;
            k_indeg_bin<<<bin_nwg, kBinT, 0, st>>>(g->col, V, E, bin_shift, bin_b, bin_nwg, binned, offt, c->d_err, bad,
                                                   qflag);
            FP_HIP(hipGetLastError());
            uint32_t split = 1;
            while (split < 16 && (size_t)bin_nwg * split * 2 <= kHistT) split *= 2;
            k_indeg_hist<<<bin_b, kHistT, (4u << bin_shift), st>>>(binned, offt, bin_nwg, split, bin_shift, V, E,
                                                                    g->row_ptr, indeg, vrec, c->d_err, bad);
            FP_HIP(hipGetLastError());
        } else {
            k_indeg_check<<<blocks_for(nmax, 256) < 8192 ? blocks_for(nmax, 256) : 8192, 256, 0, st>>>(
                g->row_ptr, g->col, V, E, indeg, c->d_err, bad, qflag);
            FP_HIP(hipGetLastError());
        }
        const uint32_t vblocks = blocks_for(V, 256);
        const unsigned eg = E ? (blocks_for(E, 256) < 8192 ? blocks_for(E, 256) : 8192) : 0u;
        k_lvl_prep<<<vblocks + eg, 256, 0, st>>>(g->has_deps, indeg, g->row_ptr, g->col, V, E, vblocks, level, state,
                                                 (uint4 *)Q, actl, erec, vrec, bad);
        FP_HIP(hipGetLastError());
        if (E) {
            k_edge_hops<<<eg, 256, 0, st>>>(E, erec, erec2, bad);
            FP_HIP(hipGetLastError());
#ifdef FP_LVL_TRACE
            {
                void *tr = nullptr;
                FP_HIP(hipGetSymbolAddress(&tr, HIP_SYMBOL(g_lvl_trace)));
                FP_HIP(hipMemsetAsync(tr, 0xFF, 4095 * 8, st));
                FP_HIP(hipMemsetAsync((char *)tr + 4095 * 8, 0, 8, st));
            }
#endif
            // one wave per block, kAsyncBlocks of them
            k_lvl_async<<<kAsyncBlocks, 64, 0, st>>>(erec, erec2, E, V, state, Q, actl, level, c->d_err, bad, qflag);
            FP_HIP(hipGetLastError());
        }
        // the cycle key (from the largest level seen) is computed on the device: no read-back; the
        // cycle count goes straight to the caller's word (zeroed by k_lvl_zero)
        const bool cs_path = counting && (((size_t)V + CS_TILE - 1) / CS_TILE) <= CS_MAX_TILES;
        if (cs_path) {
            // the counting sort reads the levels themselves (LvlMap): cycle key, keys and cycle count
            // come out of its first pass
            const LvlMap lm{actl + kMaxLevelWord, ncyc, n_cycle_dev};
            if ((rc = level_sort(st, counting, level, kb, vb, order, V, ck, bad, tmp, sort_tmp, cs_hist, c->d_err, lm))) return rc;
        } else {
            k_lvl_async_final<<<blocks_for(V, 256), 256, 0, st>>>(V, actl, level, keys, vals, ncyc, ck, bad, n_cycle_dev);
            FP_HIP(hipGetLastError());
            if ((rc = level_sort(st, counting, keys, kb, vb, order, V, ck, bad, tmp, sort_tmp, cs_hist, c->d_err))) return rc;
        }
        fp_prof_end(c, FP_K_LEVEL, ev);
        return FP_OK;
    }
    FP_HIP(hipMemsetAsync(indeg, 0, (size_t)V * 4, st));
    FP_HIP(hipMemsetAsync(cnt, 0, ncnt * 4, st));  // the per-level frontier counts
    FP_HIP(hipMemsetAsync(ncyc, 0, 64, st));
    k_check_csr<<<blocks_for(V, 256), 256, 0, st>>>(g->row_ptr, V, E, c->d_err, bad);
    FP_HIP(hipGetLastError());
    if (E) {
        k_indeg<<<blocks_for(E, 256) < 8192 ? blocks_for(E, 256) : 8192, 256, 0, st>>>(
            g->col, E, V, indeg, c->d_err, bad);
        FP_HIP(hipGetLastError());
    }
    k_lvl_init<<<blocks_for(V, 256), 256, 0, st>>>(g->has_deps, indeg, V, level, fa, &cnt[0]);
    FP_HIP(hipGetLastError());
    // corrupt CSR => stop before expanding.  This call's own `bad` word decides (read back with the
    // first frontier's size); the error itself stays in the kernel error word, reported like any
    // other (fp_ctx_sync, or the host call's copy-back), and every later kernel of the call reads
    // `bad` and does nothing -- a pending error of an earlier call is neither reported nor cleared
    FP_HIP(hipMemcpyAsync((char *)c->h_small + 8, &cnt[0], 4, hipMemcpyDeviceToHost, st));
    FP_HIP(hipMemcpyAsync((char *)c->h_small + 12, bad, 4, hipMemcpyDeviceToHost, st));
    FP_HIP(hipStreamSynchronize(st));
    const uint32_t f0 = ((uint32_t *)c->h_small)[3] ? 0u : ((uint32_t *)c->h_small)[2];
    // Levels are enqueued in chunks of kChunk launches with no read-back in between
    // (a level whose frontier is empty is a no-op launch); one read of the last
    // chunk's final counter decides whether another chunk is needed.  The grid is
    // sized for the widest possible frontier and grid-strides.
    constexpr uint32_t kChunk = 64;
    const unsigned grid = blocks_for(V, 256) < 256 ? blocks_for(V, 256) : 256;
    uint32_t L = 0;  // levels enqueued so far
    if (f0) {
        while (true) {
            for (uint32_t k = 0; k < kChunk && L + 1 < ncnt; ++k, ++L) {
                uint32_t *cur = (L & 1) ? fb : fa, *nxt = (L & 1) ? fa : fb;
                k_expand<<<grid, 256, 0, st>>>(cur, &cnt[L], g->row_ptr, g->col, level, indeg, nxt, &cnt[L + 1]);
                FP_HIP(hipGetLastError());
            }
            FP_HIP(hipMemcpyAsync(c->h_small, &cnt[L], 4, hipMemcpyDeviceToHost, st));
            FP_HIP(hipStreamSynchronize(st));
            if (((uint32_t *)c->h_small)[0] == 0 || L + 1 >= ncnt) break;
        }
    }
    const uint32_t iters = L;
    // levels <= iters + 1; cycle key sorts after every level
    const uint32_t cyc_key = iters + 2;
    k_lvl_final<<<blocks_for(V, 256), 256, 0, st>>>(indeg, V, cyc_key, level, keys, vals, ncyc, ck);
    FP_HIP(hipGetLastError());
    if ((rc = level_sort(st, counting, keys, kb, vb, order, V, ck, bad, tmp, sort_tmp, cs_hist, c->d_err))) return rc;
    if (n_cycle_dev) FP_HIP(hipMemcpyAsync(n_cycle_dev, ncyc, 4, hipMemcpyDeviceToDevice, st));
    fp_prof_end(c, FP_K_LEVEL, ev);
    return FP_OK;
}
