// fp_feas.hip -- stage 2: containers x nodes feasibility / score sweep
// (SURVEY.md 7.1 step 4, 8(d)).  Brute force over every (container, node) pair on
// the given node state; node tiles are staged in LDS and read as wave-uniform
// broadcasts while each lane owns one container.
//
// Outputs per container: first feasible node (FP_NONE if none), feasible-node
// count ("score"), and optionally the feasibility bitmap, word [(c/64)*N + n],
// bit c%64 -- exactly one wavefront ballot per node, stored coalesced.
#include "fp_internal.h"

namespace {

constexpr int kBlock = 256;   // threads per block (4 waves)
constexpr int kPer = 4;       // containers per thread: one LDS node read serves 4 x 64 containers (8: slower)
constexpr int kTile = 1024;   // nodes per LDS chunk

struct alignas(16) NodeRec {
    uint32_t cf, mf, lab, cu;  // lab holds ~labels in the LDS tile
};

struct FeasArgs {
    uint32_t C, N, WC, node_span;  // node_span: nodes per blockIdx.y (multiple of 64)
    // scenario blockIdx.z: containers/outputs advance by C per scenario, nodes by N
    // (fp_dev_feasibility_batch); 0 scenarios of stride for the single-scenario call
    const uint32_t *cpu, *mem, *req, *conf;
    const uint32_t *cf, *mf, *lab, *cu;
    const uint8_t *sched;
    uint32_t *first, *count;
    uint64_t *bitmap;
    int split;
};

// Block = 256 threads x kPer containers: container c = blockIdx.x * 1024 + k * 256 + threadIdx.x,
// so each of a wave's kPer container words is one bitmap row.
// Per (node, container) the test is two compares and ((req & ~lab) | (cu & conf)) == 0 with
// ~lab staged in LDS; unschedulable nodes are skipped with a wave-uniform branch and absent
// lanes are masked once (their count and first are never written), not per evaluation.
__global__ __launch_bounds__(kBlock) void k_feas(FeasArgs a) {
    __shared__ NodeRec rec[kTile];   // cf, mf, ~lab, cu
    __shared__ uint32_t sch[kTile];
    const uint32_t lane = threadIdx.x & 63;
    if (gridDim.z > 1) {  // scenario blockIdx.z of a batch: rebase every array on it
        const size_t sc = (size_t)blockIdx.z * a.C, sn = (size_t)blockIdx.z * a.N;
        a.cpu += sc; a.mem += sc; a.req += sc; a.conf += sc; a.first += sc; a.count += sc;
        a.cf += sn; a.mf += sn; a.lab += sn; a.cu += sn; a.sched += sn;
    }
    uint32_t cpu[kPer], mem[kPer], req[kPer], conf[kPer], first[kPer], cnt[kPer], cidx[kPer];
    uint64_t word[kPer], cinm[kPer];
    bool cin[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t c = blockIdx.x * (kBlock * kPer) + k * kBlock + threadIdx.x;
        cidx[k] = c;
        cin[k] = c < a.C;
        cpu[k] = cin[k] ? a.cpu[c] : 0xFFFFFFFFu;
        mem[k] = cin[k] ? a.mem[c] : 0xFFFFFFFFu;
        req[k] = cin[k] ? a.req[c] : 0xFFFFFFFFu;
        conf[k] = cin[k] ? a.conf[c] : 0xFFFFFFFFu;
        first[k] = FP_NONE;
        cnt[k] = 0;
        word[k] = 0;
        cinm[k] = __builtin_amdgcn_ballot_w64(cin[k]);  // absent lanes never set a bitmap bit
    }
    const uint32_t y0 = blockIdx.y * a.node_span;
    const uint32_t y1 = min(a.N, y0 + a.node_span);
    for (uint32_t n0 = y0; n0 < y1; n0 += kTile) {
        const uint32_t len = min((uint32_t)kTile, y1 - n0);
        for (uint32_t i = threadIdx.x; i < len; i += kBlock) {
            NodeRec r;
            r.cf = a.cf[n0 + i]; r.mf = a.mf[n0 + i]; r.lab = ~a.lab[n0 + i]; r.cu = a.cu[n0 + i];
            rec[i] = r;
            sch[i] = a.sched[n0 + i];
        }
        __syncthreads();
        for (uint32_t i = 0; i < len; ++i) {
            const uint32_t n = n0 + i;
            if (__builtin_amdgcn_readfirstlane(sch[i])) {
                const NodeRec r = rec[i];
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    const bool ok = (r.cf >= cpu[k]) & (r.mf >= mem[k]) & (((req[k] & r.lab) | (r.cu & conf[k])) == 0u);
                    cnt[k] += ok ? 1u : 0u;
                    first[k] = min(first[k], ok ? n : FP_NONE);
                    if (a.bitmap) {
                        const uint64_t m = __builtin_amdgcn_ballot_w64(ok) & cinm[k];  // every lane takes part
                        word[k] = lane == (i & 63) ? m : word[k];
                    }
                }
            }
            if (a.bitmap && ((i & 63) == 63 || i + 1 == len)) {
                const uint32_t nb = n0 + (i & ~63u);
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    const uint32_t wword = (blockIdx.x * (kBlock * kPer) + k * kBlock + (threadIdx.x & ~63u)) / 64;
                    if (lane <= (i & 63) && wword < a.WC) a.bitmap[(size_t)wword * a.N + nb + lane] = word[k];
                    word[k] = 0;  // skipped (unschedulable) nodes of the next 64 stay zero
                }
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (!cin[k]) continue;
        if (a.split) {
            if (first[k] != FP_NONE) atomicMin(&a.first[cidx[k]], first[k]);
            if (cnt[k]) atomicAdd(&a.count[cidx[k]], cnt[k]);
        } else {
            a.first[cidx[k]] = first[k];
            a.count[cidx[k]] = cnt[k];
        }
    }
}

}  // namespace

// Stage 2 over S what-if scenarios at once (scenario-major SoA, fp_batch): per scenario and
// container, the first feasible node and the number of feasible nodes on the scenario's node
// state.  Same kernel as the single-scenario sweep, one grid z-slice per scenario.
int fp_dev_feasibility_batch_impl(fp_ctx *c, const fp_batch *b, uint32_t *first, uint32_t *count) {
    const uint32_t S = b->n_scen, C = b->n_containers, N = b->n_nodes;
    if (S == 0 || C == 0) return FP_OK;
    if (S > 65535u) return FP_EOVERFLOW;  // grid z
    if (!b->cpu_m || !b->mem_mib || !b->req_labels || !b->conflict || !first || !count) return FP_EINVAL;
    if (N && (!b->cpu_free || !b->mem_free || !b->labels || !b->conflict_used || !b->schedulable))
        return FP_EINVAL;
    hipStream_t st = c->stream;
    const size_t SC = (size_t)S * C;
    if (N == 0) {
        FP_HIP(hipMemsetAsync(first, 0xFF, SC * 4, st));
        FP_HIP(hipMemsetAsync(count, 0, SC * 4, st));
        return FP_OK;
    }
    const uint32_t xb = (C + kBlock * kPer - 1) / (kBlock * kPer);
    // split the node range only while the whole grid is small
    uint32_t ysplit = 1;
    const uint32_t max_split = (N + 63) / 64;
    while ((uint64_t)xb * ysplit * S < 2048 && ysplit < max_split) ysplit *= 2;
    if (ysplit > max_split) ysplit = max_split;
    uint32_t span = (N + ysplit - 1) / ysplit;
    span = (span + 63) & ~63u;
    ysplit = (N + span - 1) / span;
    FeasArgs a;
    a.C = C; a.N = N; a.WC = (C + 63) / 64; a.node_span = span;
    a.cpu = b->cpu_m; a.mem = b->mem_mib; a.req = b->req_labels; a.conf = b->conflict;
    a.cf = b->cpu_free; a.mf = b->mem_free; a.lab = b->labels; a.cu = b->conflict_used;
    a.sched = b->schedulable;
    a.first = first; a.count = count; a.bitmap = nullptr;
    a.split = ysplit > 1;  // node-range splits merge with atomics into memset outputs
    if (a.split) {
        FP_HIP(hipMemsetAsync(first, 0xFF, SC * 4, st));
        FP_HIP(hipMemsetAsync(count, 0, SC * 4, st));
    }
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_FEAS, &ev);
    k_feas<<<dim3(xb, ysplit, S), kBlock, 0, st>>>(a);
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_FEAS, ev);
    return FP_OK;
}

int fp_dev_feasibility_impl(fp_ctx *c, const fp_containers *cs, const fp_nodes *ns,
                            uint32_t *first, uint32_t *count, uint64_t *bitmap) {
    const uint32_t C = cs->n, N = ns->n;
    if (C == 0) return FP_OK;
    if (!cs->cpu_m || !cs->mem_mib || !cs->req_labels || !cs->conflict || !first || !count)
        return FP_EINVAL;
    if (N && (!ns->cpu_free || !ns->mem_free || !ns->labels || !ns->conflict_used || !ns->schedulable))
        return FP_EINVAL;
    hipStream_t st = c->stream;
    const uint32_t xb = (C + kBlock * kPer - 1) / (kBlock * kPer);
    // split the node range over blockIdx.y until the grid is >= ~2048 blocks
    uint32_t ysplit = 1;
    const uint32_t max_split = N ? (N + 63) / 64 : 1;  // node ranges of >= 64 nodes
    while ((uint64_t)xb * ysplit < 2048 && ysplit < max_split) ysplit *= 2;
    if (ysplit > max_split) ysplit = max_split;
    uint32_t span = N ? (N + ysplit - 1) / ysplit : 0;
    span = (span + 63) & ~63u;
    if (span == 0) span = 64;
    ysplit = N ? (N + span - 1) / span : 1;
    FeasArgs a;
    a.C = C; a.N = N; a.WC = (C + 63) / 64; a.node_span = span;
    a.cpu = cs->cpu_m; a.mem = cs->mem_mib; a.req = cs->req_labels; a.conf = cs->conflict;
    a.cf = ns->cpu_free; a.mf = ns->mem_free; a.lab = ns->labels; a.cu = ns->conflict_used;
    a.sched = ns->schedulable;
    a.first = first; a.count = count; a.bitmap = bitmap;
    a.split = ysplit > 1;
    if (a.split || N == 0) {
        FP_HIP(hipMemsetAsync(first, 0xFF, (size_t)C * 4, st));
        FP_HIP(hipMemsetAsync(count, 0, (size_t)C * 4, st));
    }
    if (N == 0) return FP_OK;
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_FEAS, &ev);
    k_feas<<<dim3(xb, ysplit), kBlock, 0, st>>>(a);
    FP_HIP(hipGetLastError());
    fp_prof_end(c, FP_K_FEAS, ev);
    return FP_OK;
}
