// fp_gen.hip -- SPEC.md section 3 synthetic clusters generated on the device, so
// a 4096-scenario batch (3.3 GB of container records) never crosses PCIe.
// Counter-form SplitMix64: every field of every record is an independent draw,
// so each thread generates one record with no sequential state.
#include "fp_internal.h"

namespace {

__global__ void k_gen_cont(uint64_t seed, uint32_t scen_base, uint32_t S, uint32_t C, uint32_t flags,
                           uint32_t *__restrict__ cpu, uint32_t *__restrict__ mem,
                           uint32_t *__restrict__ req, uint32_t *__restrict__ conf) {
    const size_t total = (size_t)S * C;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(i / C), j = (uint32_t)(i % C);
        const uint64_t st = fpd::scenario_seed(seed, scen_base + s) ^ fpd::TAG_CONT;
        const uint64_t k = (uint64_t)j * 8;
        cpu[i] = 50u * (2u + (uint32_t)(fpd::draw(st, k + 0) % 79u));
        mem[i] = 64u * (1u + (uint32_t)(fpd::draw(st, k + 1) % 256u));
        uint32_t cf = 0, rq = 0;
        if ((flags & 1u) && fpd::draw(st, k + 2) % 1000u < 100u) cf |= 1u << (fpd::draw(st, k + 3) % 16u);
        if ((flags & 2u) && fpd::draw(st, k + 4) % 1000u < 200u)
            cf |= 1u << (16u + fpd::draw(st, k + 5) % 16u);
        if ((flags & 4u) && fpd::draw(st, k + 6) % 1000u < 300u) rq = 1u << (fpd::draw(st, k + 7) % 13u);
        conf[i] = cf;
        req[i] = rq;
    }
}

__global__ void k_gen_node(uint64_t seed, uint32_t scen_base, uint32_t S, uint32_t N,
                           uint32_t *__restrict__ cf, uint32_t *__restrict__ mf,
                           uint32_t *__restrict__ lab, uint32_t *__restrict__ cu,
                           uint8_t *__restrict__ sched) {
    const uint32_t CPU[5] = {4000, 8000, 16000, 32000, 64000};
    const uint32_t MEM[5] = {8192, 16384, 32768, 65536, 262144};
    const size_t total = (size_t)S * N;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(i / N), n = (uint32_t)(i % N);
        const uint64_t st = fpd::scenario_seed(seed, scen_base + s) ^ fpd::TAG_NODE;
        const uint64_t k = (uint64_t)n * 8;
        const uint32_t t = (uint32_t)(fpd::draw(st, k + 0) % 5u);
        cf[i] = CPU[t];
        mf[i] = MEM[t];
        uint32_t l = 0;
        l |= 1u << (0u + fpd::draw(st, k + 1) % 3u);
        l |= 1u << (3u + fpd::draw(st, k + 2) % 4u);
        l |= 1u << (7u + fpd::draw(st, k + 3) % 4u);
        l |= 1u << (11u + fpd::draw(st, k + 4) % 2u);
        lab[i] = l;
        cu[i] = 0;
        sched[i] = (fpd::draw(st, k + 5) % 1000u) >= 20u ? 1 : 0;
    }
}

inline unsigned gblocks(size_t n) {
    size_t g = (n + 255) / 256;
    if (g > 16384) g = 16384;
    return (unsigned)(g ? g : 1);
}

}  // namespace

static int gen_batch(fp_ctx *c, uint64_t seed, const fp_batch *b, uint32_t flags) {
    const size_t SC = (size_t)b->n_scen * b->n_containers, SN = (size_t)b->n_scen * b->n_nodes;
    hipEvent_t ev;
    fp_prof_begin(c, FP_K_GEN, &ev);
    if (SC) {
        if (!b->cpu_m || !b->mem_mib || !b->req_labels || !b->conflict) return FP_EINVAL;
        k_gen_cont<<<gblocks(SC), 256, 0, c->stream>>>(seed, b->scen_base, b->n_scen, b->n_containers,
                                                       flags, (uint32_t *)b->cpu_m, (uint32_t *)b->mem_mib,
                                                       (uint32_t *)b->req_labels, (uint32_t *)b->conflict);
        FP_HIP(hipGetLastError());
    }
    if (SN) {
        if (!b->cpu_free || !b->mem_free || !b->labels || !b->conflict_used || !b->schedulable)
            return FP_EINVAL;
        k_gen_node<<<gblocks(SN), 256, 0, c->stream>>>(seed, b->scen_base, b->n_scen, b->n_nodes,
                                                       b->cpu_free, b->mem_free, (uint32_t *)b->labels,
                                                       b->conflict_used, (uint8_t *)b->schedulable);
        FP_HIP(hipGetLastError());
    }
    fp_prof_end(c, FP_K_GEN, ev);
    return FP_OK;
}

extern "C" int fp_dev_gen_batch(fp_ctx *c, uint64_t seed, const fp_batch *b, uint32_t flags) {
    if (!c || !b) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_dev_done(c, gen_batch(c, seed, b, flags));
}
