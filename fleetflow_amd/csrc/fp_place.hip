// fp_place.hip -- stage 3: first-fit-decreasing placement, batched over what-if
// scenarios (SPEC.md 2.3).  One workgroup owns one scenario.
//
// Pipeline per fp_dev_place_batch call:
//   1. k_key_bounds : max(cpu_m), max(mem_mib) over the batch (exact key width)
//   2. k_make_keys  : key = ((cmax-cpu) << mb) | (mmax-mem), value = container index
//   3. rocprim segmented radix sort (stable)  => (cpu desc, mem desc, index asc)
//   4. k_ffd        : per scenario, containers in key order, lowest feasible node
//                     found by a wavefront ballot over 64-node groups; capacity
//                     updated in place by the winning lane.  Cost packed at the end.
#include "fp_internal.h"
#include <rocprim/device/device_segmented_radix_sort.hpp>

namespace {

constexpr int kWave = 64;

// out[0..1] = max(cpu), max(mem); out[2..3] = min positive cpu, mem (0xFFFFFFFF if none)
__global__ void k_key_bounds(const uint32_t *__restrict__ cpu, const uint32_t *__restrict__ mem,
                             size_t n, uint32_t *__restrict__ out /* [4] */) {
    uint32_t mc = 0, mm = 0, lc = 0xFFFFFFFFu, lm = 0xFFFFFFFFu;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t c = cpu[i], m = mem[i];
        mc = max(mc, c);
        mm = max(mm, m);
        if (c) lc = min(lc, c);
        if (m) lm = min(lm, m);
    }
    for (int o = 32; o > 0; o >>= 1) {
        mc = max(mc, (uint32_t)__shfl_xor((int)mc, o));
        mm = max(mm, (uint32_t)__shfl_xor((int)mm, o));
        lc = min(lc, (uint32_t)__shfl_xor((int)lc, o));
        lm = min(lm, (uint32_t)__shfl_xor((int)lm, o));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out[0], mc);
        atomicMax(&out[1], mm);
        atomicMin(&out[2], lc);
        atomicMin(&out[3], lm);
    }
}

__global__ void k_make_keys(const uint32_t *__restrict__ cpu, const uint32_t *__restrict__ mem,
                            size_t n, uint32_t C, uint32_t mb, uint64_t cmax, uint64_t mmax,
                            uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        keys[i] = ((cmax - cpu[i]) << mb) | (mmax - mem[i]);
        vals[i] = (uint32_t)(i % C);
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

struct FfdArgs {
    uint32_t S, C, N, scen_base;
    const uint32_t *cpu, *mem, *req, *conf, *level;
    const uint32_t *order;
    uint32_t *cf, *mf;
    const uint32_t *lab;
    uint32_t *cu;
    const uint8_t *sched;
    uint32_t *assign;
    uint8_t *reason;
    uint64_t *cost;
};

struct alignas(16) NodeRec {
    uint32_t cf, mf, cu, lab;
};

// LDS layout (kLds): NodeRec rec[NG*64] | uint64 sched[NG] | uint64 used[NG]
template <bool kLds>
__global__ __launch_bounds__(kWave) void k_ffd(FfdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t s = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const uint32_t C = a.C, N = a.N, NG = (N + kWave - 1) / kWave;
    const size_t cb = (size_t)s * C, nb = (size_t)s * N;

    // LDS: [NodeRec rec[NG*64] (kLds only)] | uint64 sched[NG] | uint64 used[NG]
    NodeRec *rec = reinterpret_cast<NodeRec *>(smem);
    uint64_t *sched = reinterpret_cast<uint64_t *>(
        smem + (kLds ? (size_t)NG * kWave * sizeof(NodeRec) : (size_t)0));
    uint64_t *used = sched + NG;

    // ---- stage node table (LDS variant) and per-group schedulable masks ----
    for (uint32_t g = 0; g < NG; ++g) {
        const uint32_t n = g * kWave + lane;
        const bool in = n < N;
        const bool sc = in && a.sched[nb + n] != 0;
        const uint64_t m = __ballot(sc);
        if (kLds) {
            NodeRec r;
            r.cf = in ? a.cf[nb + n] : 0u;
            r.mf = in ? a.mf[nb + n] : 0u;
            r.cu = in ? a.cu[nb + n] : 0u;
            r.lab = in ? a.lab[nb + n] : 0u;
            rec[n] = r;
        }
        if (lane == 0) { sched[g] = m; used[g] = 0; }
    }
    __syncthreads();

    uint32_t n_rej = 0, n_used = 0;
    for (uint32_t k0 = 0; k0 < C; k0 += kWave) {
        const uint32_t k = k0 + lane;
        const bool kin = k < C;
        const uint32_t j = kin ? a.order[cb + k] : 0u;
        const uint32_t my_cpu = kin ? a.cpu[cb + j] : 0u;
        const uint32_t my_mem = kin ? a.mem[cb + j] : 0u;
        const uint32_t my_req = kin ? a.req[cb + j] : 0u;
        const uint32_t my_conf = kin ? a.conf[cb + j] : 0u;
        const uint32_t my_cyc = (kin && a.level && a.level[cb + j] == FP_NONE) ? 1u : 0u;
        uint32_t my_assign = FP_NONE;
        uint32_t my_reason = FP_REASON_OK;
        const uint32_t cnt = min((uint32_t)kWave, C - k0);
        for (uint32_t t = 0; t < cnt; ++t) {
            const uint32_t ccpu = __builtin_amdgcn_readlane(my_cpu, t);
            const uint32_t cmem = __builtin_amdgcn_readlane(my_mem, t);
            const uint32_t creq = __builtin_amdgcn_readlane(my_req, t);
            const uint32_t cconf = __builtin_amdgcn_readlane(my_conf, t);
            const uint32_t ccyc = __builtin_amdgcn_readlane(my_cyc, t);
            uint32_t hit = FP_NONE;
            if (!ccyc) {
                for (uint32_t g = 0; g < NG; ++g) {
                    const uint32_t n = g * kWave + lane;
                    uint32_t cf, mf, cu, lab;
                    if (kLds) {
                        const NodeRec r = rec[n];
                        cf = r.cf; mf = r.mf; cu = r.cu; lab = r.lab;
                    } else {
                        const bool in = n < N;
                        // sc1 loads: this wave's own earlier stores must be observed
                        cf = in ? __hip_atomic_load(&a.cf[nb + n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                        mf = in ? __hip_atomic_load(&a.mf[nb + n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                        cu = in ? __hip_atomic_load(&a.cu[nb + n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                        lab = in ? a.lab[nb + n] : 0u;
                    }
                    const bool ok = fpd::fits(ccpu, cmem, creq, cconf, cf, mf, lab, cu);
                    const uint64_t m = __ballot(ok) & sched[g];
                    if (m) {
                        const uint32_t l = (uint32_t)__builtin_ctzll(m);
                        hit = g * kWave + l;
                        if (lane == l) {
                            if (kLds) {
                                NodeRec r;
                                r.cf = cf - ccpu; r.mf = mf - cmem; r.cu = cu | cconf; r.lab = lab;
                                rec[n] = r;
                            } else {
                                __hip_atomic_store(&a.cf[nb + n], cf - ccpu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                __hip_atomic_store(&a.mf[nb + n], mf - cmem, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                __hip_atomic_store(&a.cu[nb + n], cu | cconf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            }
                        }
                        const uint64_t um = used[g];
                        if (!((um >> l) & 1ull)) {
                            n_used++;
                            if (lane == 0) used[g] = um | (1ull << l);
                        }
                        break;
                    }
                }
                if (hit == FP_NONE) n_rej++;
            } else {
                n_rej++;
            }
            if (lane == t) {
                my_assign = hit;
                my_reason = ccyc ? FP_REASON_CYCLE : (hit == FP_NONE ? FP_REASON_NOFIT : FP_REASON_OK);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (kin) {
            a.assign[cb + j] = my_assign;
            a.reason[cb + j] = (uint8_t)my_reason;
        }
    }

    // ---- write the mutated node state back (LDS variant) ----
    if (kLds) {
        __syncthreads();
        for (uint32_t n = lane; n < N; n += kWave) {
            const NodeRec r = rec[n];
            a.cf[nb + n] = r.cf;
            a.mf[nb + n] = r.mf;
            a.cu[nb + n] = r.cu;
        }
    }
    if (lane == 0 && a.cost) a.cost[s] = fpd::pack_cost(n_rej, n_used, a.scen_base + s);
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

static inline unsigned grid_for(size_t n, unsigned block) {
    size_t g = (n + block - 1) / block;
    if (g > 65535u * 4) g = 65535u * 4;
    return (unsigned)(g ? g : 1);
}

int fp_dev_place_batch_impl(fp_ctx *c, const fp_batch *b) {
    const uint32_t S = b->n_scen, C = b->n_containers, N = b->n_nodes;
    if (S == 0 || C == 0) return FP_OK;
    const size_t SC = (size_t)S * C;
    if (SC > 0xFFFFFFFFull) return FP_EOVERFLOW;  // rocprim segmented sort takes u32 sizes
    if (!b->cpu_m || !b->mem_mib || !b->req_labels || !b->conflict || !b->assign || !b->reason)
        return FP_EINVAL;
    if (N && (!b->cpu_free || !b->mem_free || !b->labels || !b->conflict_used || !b->schedulable))
        return FP_EINVAL;
    hipStream_t st = c->stream;
    FP_HIP(hipMemsetAsync(c->d_err, 0, 4, st));

    const uint32_t NG = (N + kWave - 1) / kWave;
    // ---- workspace ----
    size_t sort_tmp = 0;
    FP_HIP(rocprim::segmented_radix_sort_pairs(nullptr, sort_tmp, (uint64_t *)nullptr,
                                               (uint64_t *)nullptr, (uint32_t *)nullptr,
                                               (uint32_t *)nullptr, (unsigned)SC, S,
                                               (uint32_t *)nullptr, (uint32_t *)nullptr, 0, 64, st));
    const size_t need = SC * (8 * 2 + 4 * 2 + 4 * 5) + (S + 1) * 4 + sort_tmp + 24 * 256;
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
    if (!keys_in || !keys_out || !vals_in || !vals_out || !offs || !tmp || !bounds)
        return FP_ENOMEM;

    // ---- 1-3: FFD order ----
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_SORT, &ev);
    FP_HIP(hipMemsetAsync(bounds, 0, 8, st));
    FP_HIP(hipMemsetAsync(bounds + 2, 0xFF, 8, st));
    k_key_bounds<<<grid_for(SC, 256) < 1024 ? grid_for(SC, 256) : 1024, 256, 0, st>>>(
        b->cpu_m, b->mem_mib, SC, bounds);
    FP_HIP(hipGetLastError());
    FP_HIP(hipMemcpyAsync(c->h_small, bounds, 16, hipMemcpyDeviceToHost, st));
    FP_HIP(hipStreamSynchronize(st));
    const uint32_t maxc = ((uint32_t *)c->h_small)[0], maxm = ((uint32_t *)c->h_small)[1];
    const uint32_t minc = ((uint32_t *)c->h_small)[2], minm = ((uint32_t *)c->h_small)[3];
    const uint32_t cbits = fp_bitwidth(maxc), mbits = fp_bitwidth(maxm);
    const uint32_t kbits = cbits + mbits;
    const uint64_t cmax = cbits ? ((cbits == 64 ? ~0ull : ((1ull << cbits) - 1))) : 0ull;
    const uint64_t mmax = mbits ? ((1ull << mbits) - 1) : 0ull;
    const uint32_t *order = nullptr;
    if (kbits == 0) {
        k_iota_vals<<<grid_for(SC, 256), 256, 0, st>>>(SC, C, vals_out);
        FP_HIP(hipGetLastError());
        order = vals_out;
    } else {
        k_make_keys<<<grid_for(SC, 256), 256, 0, st>>>(b->cpu_m, b->mem_mib, SC, C, mbits, cmax,
                                                       mmax, keys_in, vals_in);
        FP_HIP(hipGetLastError());
        k_seg_offsets<<<(S + 1 + 255) / 256, 256, 0, st>>>(S, C, offs);
        FP_HIP(hipGetLastError());
        FP_HIP(rocprim::segmented_radix_sort_pairs(tmp, sort_tmp, keys_in, keys_out, vals_in,
                                                   vals_out, (unsigned)SC, S, offs, offs + 1, 0,
                                                   kbits, st));
        order = vals_out;
    }
    fp_prof_end(c, FP_K_SORT, ev);

    // ---- 4: placement ----
    uint32_t pG, pW;
    size_t plds;
    if (fp_pipe_plan(N, &pG, &pW, &plds))
        return fp_pipe_launch(c, S, C, N, b->scen_base, order, b, minc == 0xFFFFFFFFu ? 1u : minc, maxc,
                              minm == 0xFFFFFFFFu ? 1u : minm, maxm);
    FfdArgs a;
    a.S = S; a.C = C; a.N = N; a.scen_base = b->scen_base;
    a.cpu = b->cpu_m; a.mem = b->mem_mib; a.req = b->req_labels; a.conf = b->conflict;
    a.level = b->level; a.order = order;
    a.cf = b->cpu_free; a.mf = b->mem_free; a.lab = b->labels; a.cu = b->conflict_used;
    a.sched = b->schedulable; a.assign = b->assign; a.reason = b->reason; a.cost = b->cost;
    const size_t lds_full = (size_t)NG * kWave * sizeof(NodeRec) + (size_t)NG * 16;
    const size_t lds_limit = 150 * 1024;
    fp_prof_begin(c, FP_K_PLACE, &ev);
    if (lds_full <= lds_limit) {
        if (lds_full > 64 * 1024)
            FP_HIP(hipFuncSetAttribute((const void *)k_ffd<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_full));
        k_ffd<true><<<S, kWave, lds_full, st>>>(a);
    } else {
        const size_t lds_small = (size_t)NG * 16;
        if (lds_small > lds_limit) return FP_EOVERFLOW;
        if (lds_small > 64 * 1024)
            FP_HIP(hipFuncSetAttribute((const void *)k_ffd<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_small));
        k_ffd<false><<<S, kWave, lds_small, st>>>(a);
    }
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_PLACE, ev);
    return FP_OK;
}

extern "C" int fp_dev_argmin_cost(fp_ctx *c, const uint64_t *cost, uint32_t n, uint32_t *best) {
    if (!c || !cost || !best || n == 0) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    k_argmin_cost<<<1, 1024, 0, c->stream>>>(cost, n, best);
    FP_HIP(hipGetLastError());
    return FP_OK;
}
