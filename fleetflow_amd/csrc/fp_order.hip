// fp_order.hip -- stage 1: start ordering.
//
//  * fp_dev_legacy_order: crates/fleetflow-container/src/engine.rs:67-85 as a stable
//    two-bucket partition (has_deps == 0 first, each bucket in input order),
//    computed with wavefront ballots + a block-offset scan.
//  * fp_dev_levelize: SPEC.md 2.2, frontier-parallel Kahn over the reversed CSR.
//    level(v) = max(has_deps(v), max_{d->v} level(d)+1) is unique, so the frontier
//    schedule (atomic order inside a level) cannot change the result.
#include "fp_internal.h"
#include <rocprim/device/device_radix_sort.hpp>

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
__global__ void k_check_csr(const uint32_t *__restrict__ row_ptr, uint32_t V, uint32_t E,
                            uint32_t *__restrict__ err) {
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) {
        if (row_ptr[v + 1] < row_ptr[v]) atomicMax(err, (uint32_t)(-FP_ECORRUPT));
    }
    if (v == 0 && (row_ptr[0] != 0 || row_ptr[V] != E)) atomicMax(err, (uint32_t)(-FP_ECORRUPT));
}

__global__ void k_indeg(const uint32_t *__restrict__ col, uint32_t E, uint32_t V,
                        uint32_t *__restrict__ indeg, uint32_t *__restrict__ err) {
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
         e += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = col[e];
        if (v >= V) atomicMax(err, (uint32_t)(-FP_ECORRUPT));
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
                            uint32_t *__restrict__ level, uint32_t *__restrict__ keys,
                            uint32_t *__restrict__ vals, uint32_t *__restrict__ ncyc) {
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
    FP_HIP(hipMemsetAsync(c->d_err, 0, 4, st));
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
    FP_HIP(hipMemsetAsync(c->d_err, 0, 4, st));

    size_t sort_tmp = 0;
    FP_HIP(rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                     (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)V, 0, 32, st));
    // cnt[L] = frontier size of level L (one counter per possible level: <= V + 1)
    const size_t ncnt = (size_t)V + 2;
    int rc = fp_ws_reserve(c, (size_t)V * 4 * 6 + ncnt * 4 + sort_tmp + 16 * 256);
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
    if (!indeg || !fa || !fb || !keys || !keys_out || !vals || !cnt || !ncyc || !tmp) return FP_ENOMEM;

    hipEvent_t ev;
    fp_prof_begin(c, FP_K_LEVEL, &ev);
    FP_HIP(hipMemsetAsync(indeg, 0, (size_t)V * 4, st));
    FP_HIP(hipMemsetAsync(cnt, 0, ncnt * 4, st));
    FP_HIP(hipMemsetAsync(ncyc, 0, 64, st));
    k_check_csr<<<blocks_for(V, 256), 256, 0, st>>>(g->row_ptr, V, E, c->d_err);
    FP_HIP(hipGetLastError());
    if (E) {
        k_indeg<<<blocks_for(E, 256) < 8192 ? blocks_for(E, 256) : 8192, 256, 0, st>>>(
            g->col, E, V, indeg, c->d_err);
        FP_HIP(hipGetLastError());
    }
    k_lvl_init<<<blocks_for(V, 256), 256, 0, st>>>(g->has_deps, indeg, V, level, fa, &cnt[0]);
    FP_HIP(hipGetLastError());
    // corrupt CSR => stop before expanding
    FP_HIP(hipMemcpyAsync(c->h_small, c->d_err, 4, hipMemcpyDeviceToHost, st));
    FP_HIP(hipMemcpyAsync((char *)c->h_small + 8, &cnt[0], 4, hipMemcpyDeviceToHost, st));
    FP_HIP(hipStreamSynchronize(st));
    if (((uint32_t *)c->h_small)[0]) return -(int)((uint32_t *)c->h_small)[0];
    const uint32_t f0 = ((uint32_t *)c->h_small)[2];
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
    k_lvl_final<<<blocks_for(V, 256), 256, 0, st>>>(indeg, V, cyc_key, level, keys, vals, ncyc);
    FP_HIP(hipGetLastError());
    FP_HIP(rocprim::radix_sort_pairs(tmp, sort_tmp, keys, keys_out, vals, order, (size_t)V, 0,
                                     fp_bitwidth(cyc_key), st));
    if (n_cycle_dev) FP_HIP(hipMemcpyAsync(n_cycle_dev, ncyc, 4, hipMemcpyDeviceToDevice, st));
    fp_prof_end(c, FP_K_LEVEL, ev);
    return FP_OK;
}
