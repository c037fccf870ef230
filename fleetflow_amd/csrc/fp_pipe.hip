// fp_pipe.hip -- stage 3 FFD as an intra-workgroup tile pipeline (SPEC.md 2.3).
//
// One workgroup = one scenario.  Its N nodes are cut into W tiles of G x 64 nodes;
// wave w owns tile w with the node state (cpu_free, mem_free, conflict_used,
// labels) RESIDENT IN VGPRs (lane l of group g holds node w*G*64 + g*64 + l).
// Containers stream through the waves in FFD order: wave 0 reads the sorted
// container list from HBM, places what fits its tile (lowest node first) and
// forwards the rest, in order, to wave 1 through an LDS ring, and so on; what
// the last wave cannot place is NOFIT.
//
// Exactness: a container lands in the first tile holding a feasible node, and a
// tile's state only depends on the containers that reached it, in FFD order --
// so the pipeline computes exactly the sequential first fit.
//
// Pruning (exact): per tile, per 64-node group g and per threshold bucket k, two
// 64-bit masks  B_cpu[g][k] = {l : sched && cpu_free >= Tc[k]} and
// B_mem[g][k] = {l : sched && mem_free >= Tm[k]}  live in LDS.  A container with
// bucket indices (kc, km) (Tc[kc] <= cpu, Tm[km] <= mem) can only fit nodes in
// B_cpu[g][kc] & B_mem[g][km]; free capacity only shrinks (SPEC.md 2.3
// monotonicity), so masks are maintained by clearing bits on placement and a
// stale mask is always a superset.  Only candidate groups get the exact
// register-resident check.
#include "fp_internal.h"

namespace fpp {

constexpr int K = 32;               // threshold buckets per dimension
constexpr int R = 4;                // LDS ring slots per link
constexpr uint32_t END = 0x80000000u;
constexpr uint32_t CYC = 0x80000000u;
constexpr uint32_t SPIN_LIMIT = 1u << 26;

struct PipeArgs {
    uint32_t C, N, scen_base, W;
    const uint32_t *s_cpu, *s_mem, *s_req, *s_conf, *s_idx;  // FFD-sorted SoA [S][C]; idx bit31 = CYCLE
    uint32_t *cf, *mf;
    const uint32_t *lab;
    uint32_t *cu;
    const uint8_t *sched;
    uint32_t *assign;
    uint8_t *reason;
    uint64_t *cost;
    uint32_t *err;
    uint32_t tc[K], tm[K];  // ascending thresholds, tc[0] = tm[0] = 0
};

__device__ __forceinline__ uint32_t lds_acq(uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_rel(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int G>
struct Tile {
    uint32_t cf[G], mf[G], cu[G], lab[G];
};

// Exact check of group g (compile-time) for the wave-uniform container; on a hit
// the winning lane's node is updated in registers and the LDS masks are cleared.
template <int G, int g>
__device__ __forceinline__ bool check_group(Tile<G> &t, uint64_t *Mg, uint64_t *Ug, uint32_t lane,
                                            uint32_t c_cpu, uint32_t c_mem, uint32_t c_req, uint32_t c_conf,
                                            uint32_t c_kc, uint32_t c_km, uint32_t my_tc, uint32_t my_tm,
                                            uint32_t &n_used, uint32_t &node) {
    const uint64_t wm = Mg[c_kc * 2] & Mg[c_km * 2 + 1];
    const bool ok = fpd::fits(c_cpu, c_mem, c_req, c_conf, t.cf[g], t.mf[g], t.lab[g], t.cu[g]);
    const uint64_t m = __ballot(ok) & wm;
    if (!m) return false;
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    const uint32_t oc = __builtin_amdgcn_readlane(t.cf[g], l);
    const uint32_t om = __builtin_amdgcn_readlane(t.mf[g], l);
    const uint32_t nc = oc - c_cpu, nm = om - c_mem;
    if (lane == l) {
        t.cf[g] = nc;
        t.mf[g] = nm;
        t.cu[g] |= c_conf;
    }
    if (lane < (uint32_t)K) {
        const uint64_t clr = ~(1ull << l);
        if (my_tc <= oc && my_tc > nc) atomicAnd((unsigned long long *)&Mg[lane * 2], (unsigned long long)clr);
        if (my_tm <= om && my_tm > nm) atomicAnd((unsigned long long *)&Mg[lane * 2 + 1], (unsigned long long)clr);
    }
    const uint64_t u = *Ug;
    if (!((u >> l) & 1ull)) {
        n_used++;
        if (lane == 0) *Ug = u | (1ull << l);
    }
    node = (uint32_t)g * 64u + l;
    return true;
}

// Balanced dispatch over candidate group gi in [LO, HI) to the compile-time check.
template <int G, int LO, int HI>
__device__ __forceinline__ bool dispatch(uint32_t gi, Tile<G> &t, uint64_t *M, uint64_t *U, uint32_t lane,
                                         uint32_t c_cpu, uint32_t c_mem, uint32_t c_req, uint32_t c_conf,
                                         uint32_t c_kc, uint32_t c_km, uint32_t my_tc, uint32_t my_tm,
                                         uint32_t &n_used, uint32_t &node) {
    if constexpr (HI - LO == 1) {
        return check_group<G, LO>(t, M + (size_t)LO * K * 2, U + LO, lane, c_cpu, c_mem, c_req, c_conf, c_kc,
                                  c_km, my_tc, my_tm, n_used, node);
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (gi < (uint32_t)MID)
            return dispatch<G, LO, MID>(gi, t, M, U, lane, c_cpu, c_mem, c_req, c_conf, c_kc, c_km, my_tc, my_tm,
                                        n_used, node);
        return dispatch<G, MID, HI>(gi, t, M, U, lane, c_cpu, c_mem, c_req, c_conf, c_kc, c_km, my_tc, my_tm,
                                    n_used, node);
    }
}

// Spin on an LDS word until pred holds; bounded, with a workgroup abort flag.
template <class Pred>
__device__ __forceinline__ bool spin(uint32_t *word, Pred pred, uint32_t *abort_flag, uint32_t *err) {
    uint32_t n = 0;
    while (true) {
        const uint32_t v = lds_acq(word);
        if (pred(v)) return true;
        if (lds_acq(abort_flag)) return false;
        if (++n > SPIN_LIMIT) {
            lds_rel(abort_flag, 1u);
            if ((threadIdx.x & 63) == 0) atomicMax(err, (uint32_t)(-FP_EDEVICE));
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// LDS layout (bytes, all offsets 16-aligned):
//   M   : W*G*K*2 u64   (B_cpu, B_mem interleaved per (g, k))
//   U   : W*G u64       (node-used masks)
//   CTL : (W-1)*8 u32   per link: [0]=head [1]=tail [2..2+R)=slot counts
//   CNT : 8 u32         [0]=n_used [1]=n_rej [2]=abort
//   D   : (W-1)*R*6*64 u32 ring data (cpu, mem, req, conf, idx, kk) per slot
template <int G, int MAXW>
__global__ __launch_bounds__(MAXW * 64) void k_ffd_pipe(const PipeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t W = a.W;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t s = blockIdx.x;
    const uint32_t C = a.C, N = a.N;
    const size_t cb = (size_t)s * C, nb = (size_t)s * N;

    uint64_t *M = reinterpret_cast<uint64_t *>(smem);
    uint64_t *U = M + (size_t)W * G * K * 2;
    uint32_t *CTL = reinterpret_cast<uint32_t *>(U + (size_t)W * G);
    uint32_t *CNT = CTL + (W - 1) * 8;
    uint32_t *D = CNT + 8;

    for (uint32_t i = threadIdx.x; i < (W - 1) * 8 + 8; i += blockDim.x) CTL[i] = 0;

    // ---- load the tile into VGPRs and build the bucket masks ----
    const uint32_t my_tc = lane < (uint32_t)K ? a.tc[lane] : 0xFFFFFFFFu;
    const uint32_t my_tm = lane < (uint32_t)K ? a.tm[lane] : 0xFFFFFFFFu;
    const uint32_t nbase = w * G * 64;
    Tile<G> t;
    uint64_t *Mw = M + (size_t)w * G * K * 2;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint32_t n = nbase + g * 64 + lane;
        const bool in = n < N;
        const bool sc = in && a.sched[nb + n] != 0;
        t.cf[g] = in ? a.cf[nb + n] : 0u;
        t.mf[g] = in ? a.mf[nb + n] : 0u;
        t.cu[g] = in ? a.cu[nb + n] : 0u;
        t.lab[g] = in ? a.lab[nb + n] : 0u;
#pragma unroll 1
        for (int k = 0; k < K; ++k) {
            const uint32_t tck = __builtin_amdgcn_readlane(my_tc, k);
            const uint32_t tmk = __builtin_amdgcn_readlane(my_tm, k);
            const uint64_t bc = __ballot(sc && t.cf[g] >= tck);
            const uint64_t bm = __ballot(sc && t.mf[g] >= tmk);
            if (lane == 0) {
                Mw[((size_t)g * K + k) * 2] = bc;
                Mw[((size_t)g * K + k) * 2 + 1] = bm;
            }
        }
        if (lane == 0) U[(size_t)w * G + g] = 0;
    }
    __syncthreads();

    const bool has_out = w + 1 < W;
    uint32_t *octl = CTL + w * 8;
    uint32_t *ictl = CTL + (w - 1) * 8;
    uint32_t *odata = D + (size_t)w * R * 6 * 64;
    uint32_t *idata = D + (size_t)(w - 1) * R * 6 * 64;
    uint32_t *abort_flag = &CNT[2];
    uint32_t ohead = 0, ofill = 0, itail = 0, k0 = 0;
    uint32_t n_used = 0, n_rej = 0;
    bool alive = true;

    while (alive) {
        uint32_t cpu = 0, mem = 0, req = 0, conf = 0, idx = 0, kk = 0;
        bool valid = false;
        if (w == 0) {
            if (k0 >= C) break;
            const uint32_t i = k0 + lane;
            valid = i < C;
            if (valid) {
                cpu = a.s_cpu[cb + i];
                mem = a.s_mem[cb + i];
                req = a.s_req[cb + i];
                conf = a.s_conf[cb + i];
                idx = a.s_idx[cb + i];
            }
            const bool cyc = valid && (idx & CYC);
            if (cyc) {
                const uint32_t j = idx & ~CYC;
                a.assign[cb + j] = FP_NONE;
                a.reason[cb + j] = FP_REASON_CYCLE;
            }
            n_rej += (uint32_t)__popcll(__ballot(cyc));
            valid = valid && !cyc;
            uint32_t kc = 0, km = 0;
            for (int k = 1; k < K; ++k) {
                kc += cpu >= __builtin_amdgcn_readlane(my_tc, k) ? 1u : 0u;
                km += mem >= __builtin_amdgcn_readlane(my_tm, k) ? 1u : 0u;
            }
            kk = kc | (km << 8);
            k0 += 64;
        } else {
            const uint32_t want = itail;
            if (!spin(&ictl[0], [want](uint32_t h) { return h != want; }, abort_flag, a.err)) break;
            const uint32_t slot = itail % R;
            const uint32_t n = ictl[2 + slot];
            if (n & END) break;
            const uint32_t *sd = idata + (size_t)slot * 6 * 64;
            valid = lane < n;
            if (valid) {
                cpu = sd[lane];
                mem = sd[64 + lane];
                req = sd[128 + lane];
                conf = sd[192 + lane];
                idx = sd[256 + lane];
                kk = sd[320 + lane];
            }
            itail++;
            lds_rel(&ictl[1], itail);
        }
        const uint32_t kc = kk & 0xFFu, km = kk >> 8;

        // lane-parallel candidate groups (superset; masks only lose bits)
        uint32_t cand = 0;
        if (valid) {
#pragma unroll 4
            for (int g = 0; g < G; ++g) {
                const uint64_t *mg = Mw + (size_t)g * K * 2;
                if (mg[kc * 2] & mg[km * 2 + 1]) cand |= 1u << g;
            }
        }
        uint64_t todo = __ballot(cand != 0);
        uint64_t placed = 0;
        uint32_t my_assign = FP_NONE;
        while (todo) {
            const uint32_t ti = (uint32_t)__builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t c_cpu = __builtin_amdgcn_readlane(cpu, ti);
            const uint32_t c_mem = __builtin_amdgcn_readlane(mem, ti);
            const uint32_t c_req = __builtin_amdgcn_readlane(req, ti);
            const uint32_t c_conf = __builtin_amdgcn_readlane(conf, ti);
            const uint32_t c_kk = __builtin_amdgcn_readlane(kk, ti);
            uint32_t cc = __builtin_amdgcn_readlane(cand, ti);
            const uint32_t c_kc = c_kk & 0xFFu, c_km = c_kk >> 8;
            while (cc) {
                const uint32_t gi = (uint32_t)__builtin_ctz(cc);
                cc &= cc - 1;
                uint32_t node = 0;
                if (dispatch<G, 0, G>(gi, t, Mw, U + (size_t)w * G, lane, c_cpu, c_mem, c_req, c_conf, c_kc, c_km,
                                      my_tc, my_tm, n_used, node)) {
                    placed |= 1ull << ti;
                    if (lane == ti) my_assign = nbase + node;
                    break;
                }
            }
        }
        if ((placed >> lane) & 1ull) {
            a.assign[cb + idx] = my_assign;
            a.reason[cb + idx] = FP_REASON_OK;
        }
        const bool fwd = valid && !((placed >> lane) & 1ull);
        if (!has_out) {
            if (fwd) {
                a.assign[cb + idx] = FP_NONE;
                a.reason[cb + idx] = FP_REASON_NOFIT;
            }
            n_rej += (uint32_t)__popcll(__ballot(fwd));
            continue;
        }
        const uint64_t fm = __ballot(fwd);
        const uint32_t f = (uint32_t)__popcll(fm);
        if (!f) continue;
        const uint32_t pos = ofill + (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
        uint32_t *od = odata + (size_t)(ohead % R) * 6 * 64;
        if (fwd && pos < 64) {
            od[pos] = cpu; od[64 + pos] = mem; od[128 + pos] = req;
            od[192 + pos] = conf; od[256 + pos] = idx; od[320 + pos] = kk;
        }
        if (ofill + f >= 64) {
            octl[2 + ohead % R] = 64;
            ohead++;
            lds_rel(&octl[0], ohead);
            const uint32_t h = ohead;
            if (!spin(&octl[1], [h](uint32_t tl) { return h - tl < (uint32_t)R; }, abort_flag, a.err)) {
                alive = false;
                break;
            }
            od = odata + (size_t)(ohead % R) * 6 * 64;
            if (fwd && pos >= 64) {
                const uint32_t p = pos - 64;
                od[p] = cpu; od[64 + p] = mem; od[128 + p] = req;
                od[192 + p] = conf; od[256 + p] = idx; od[320 + p] = kk;
            }
            ofill = ofill + f - 64;
        } else {
            ofill += f;
        }
    }

    // ---- flush + end of stream ----
    if (has_out && !lds_acq(abort_flag)) {
        bool ok = true;
        if (ofill) {
            octl[2 + ohead % R] = ofill;
            ohead++;
            lds_rel(&octl[0], ohead);
            const uint32_t h = ohead;
            ok = spin(&octl[1], [h](uint32_t tl) { return h - tl < (uint32_t)R; }, abort_flag, a.err);
        }
        if (ok) {
            octl[2 + ohead % R] = END;
            ohead++;
            lds_rel(&octl[0], ohead);
        }
    }
    if (lane == 0) {
        atomicAdd(&CNT[0], n_used);
        atomicAdd(&CNT[1], n_rej);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint32_t n = nbase + g * 64 + lane;
        if (n < N) {
            a.cf[nb + n] = t.cf[g];
            a.mf[nb + n] = t.mf[g];
            a.cu[nb + n] = t.cu[g];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && a.cost) a.cost[s] = fpd::pack_cost(CNT[1], CNT[0], a.scen_base + s);
}

__global__ void k_gather_sorted(uint32_t S, uint32_t C, const uint32_t *__restrict__ order,
                                const uint32_t *__restrict__ cpu, const uint32_t *__restrict__ mem,
                                const uint32_t *__restrict__ req, const uint32_t *__restrict__ conf,
                                const uint32_t *__restrict__ level, uint32_t *__restrict__ s_cpu,
                                uint32_t *__restrict__ s_mem, uint32_t *__restrict__ s_req,
                                uint32_t *__restrict__ s_conf, uint32_t *__restrict__ s_idx) {
    const size_t total = (size_t)S * C;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const size_t base = i - i % C;
        const uint32_t j = order[i];
        const size_t src = base + j;
        s_cpu[i] = cpu[src];
        s_mem[i] = mem[src];
        s_req[i] = req[src];
        s_conf[i] = conf[src];
        s_idx[i] = j | ((level && level[src] == FP_NONE) ? CYC : 0u);
    }
}

size_t lds_bytes(uint32_t W, uint32_t G) {
    return (size_t)W * G * K * 16 + (size_t)W * G * 8 + ((size_t)(W - 1) * 8 + 8) * 4 +
           (size_t)(W - 1) * R * 6 * 64 * 4;
}

}  // namespace fpp

using namespace fpp;

static const int kGs[] = {2, 4, 8, 12, 16, 20, 24, 32};

// Largest workgroup (in waves) instantiated for a tile of G groups: VGPR budget
// is 512 / (waves per SIMD), and the tile alone takes 4*G VGPRs.
static inline uint32_t max_waves_for(int G) { return G <= 4 ? 16u : (G <= 24 ? 8u : 4u); }

// Picks (G, W) for NG groups; returns false when the tile pipeline cannot host N.
bool fp_pipe_plan(uint32_t N, uint32_t *G_out, uint32_t *W_out, size_t *lds_out) {
    const uint32_t NG = (N + 63) / 64;
    if (NG == 0) {
        *G_out = 2; *W_out = 1; *lds_out = lds_bytes(1, 2);
        return true;
    }
    for (uint32_t wmax : {4u, 8u, 16u}) {
        for (int G : kGs) {
            const uint32_t W = (NG + G - 1) / G;
            if (W > wmax || W > max_waves_for(G)) continue;
            const size_t lds = lds_bytes(W, G);
            if (lds > 160 * 1024) continue;
            *G_out = G; *W_out = W; *lds_out = lds;
            return true;
        }
    }
    return false;
}

int fp_pipe_launch(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, uint32_t scen_base, const uint32_t *order,
                   const fp_batch *b, uint32_t maxc, uint32_t maxm) {
    uint32_t G, W;
    size_t lds;
    if (!fp_pipe_plan(N, &G, &W, &lds)) return FP_EOVERFLOW;
    if (C >= 0x80000000u) return FP_EOVERFLOW;
    hipStream_t st = c->stream;
    const size_t SC = (size_t)S * C;
    uint32_t *s_cpu = (uint32_t *)fp_ws_take(c, SC * 4);
    uint32_t *s_mem = (uint32_t *)fp_ws_take(c, SC * 4);
    uint32_t *s_req = (uint32_t *)fp_ws_take(c, SC * 4);
    uint32_t *s_conf = (uint32_t *)fp_ws_take(c, SC * 4);
    uint32_t *s_idx = (uint32_t *)fp_ws_take(c, SC * 4);
    if (!s_cpu || !s_mem || !s_req || !s_conf || !s_idx) return FP_ENOMEM;
    {
        size_t g = (SC + 255) / 256;
        if (g > 16384) g = 16384;
        k_gather_sorted<<<(unsigned)g, 256, 0, st>>>(S, C, order, b->cpu_m, b->mem_mib, b->req_labels, b->conflict,
                                                    b->level, s_cpu, s_mem, s_req, s_conf, s_idx);
        FP_HIP(hipGetLastError());
    }
    PipeArgs a;
    a.C = C; a.N = N; a.scen_base = scen_base; a.W = W;
    a.s_cpu = s_cpu; a.s_mem = s_mem; a.s_req = s_req; a.s_conf = s_conf; a.s_idx = s_idx;
    a.cf = b->cpu_free; a.mf = b->mem_free; a.lab = b->labels; a.cu = b->conflict_used; a.sched = b->schedulable;
    a.assign = b->assign; a.reason = b->reason; a.cost = b->cost; a.err = c->d_err;
    // thresholds: T0 = 0, then quarter-octave steps up to the batch maximum
    a.tc[0] = 0; a.tm[0] = 0;
    for (int k = 1; k < K; ++k) {
        const double e = -(double)(K - 1 - k) / 4.0;
        uint32_t vc = (uint32_t)ceil((double)maxc * pow(2.0, e));
        uint32_t vm = (uint32_t)ceil((double)maxm * pow(2.0, e));
        a.tc[k] = vc > a.tc[k - 1] ? vc : a.tc[k - 1];
        a.tm[k] = vm > a.tm[k - 1] ? vm : a.tm[k - 1];
    }
    // instantiation: smallest MAXW bucket (4, 8, 16) that holds W waves
    const uint32_t MW = W <= 4 ? 4 : (W <= 8 ? 8 : 16);
    const void *fn = nullptr;
#define FP_PIPE_CASE(GG, MM) \
    if (G == GG && MW == MM) fn = (const void *)k_ffd_pipe<GG, MM>;
    FP_PIPE_CASE(2, 4) FP_PIPE_CASE(2, 8) FP_PIPE_CASE(2, 16)
    FP_PIPE_CASE(4, 4) FP_PIPE_CASE(4, 8) FP_PIPE_CASE(4, 16)
    FP_PIPE_CASE(8, 4) FP_PIPE_CASE(8, 8)
    FP_PIPE_CASE(12, 4) FP_PIPE_CASE(12, 8)
    FP_PIPE_CASE(16, 4) FP_PIPE_CASE(16, 8)
    FP_PIPE_CASE(20, 4) FP_PIPE_CASE(20, 8)
    FP_PIPE_CASE(24, 4) FP_PIPE_CASE(24, 8)
    FP_PIPE_CASE(32, 4)
#undef FP_PIPE_CASE
    if (!fn) return FP_EINVAL;
    FP_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_PLACE, &ev);
    void *kargs[] = {(void *)&a};
    FP_HIP(hipLaunchKernel(fn, dim3(S), dim3(W * 64), kargs, lds, st));
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_PLACE, ev);
    return FP_OK;
}
