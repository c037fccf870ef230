// fp_internal.h -- shared internals of libfleetplace.so (HIP, gfx950 only).
#pragma once
#include <cmath>
#include <cstring>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>
#include "../../include/fleetplace.h"

#define FP_HIP(call)                                   \
    do {                                               \
        hipError_t e_ = (call);                        \
        if (e_ != hipSuccess) return fp_hip_fail(e_);  \
    } while (0)

int fp_hip_fail(hipError_t e);

// A word that only gains bits (the batch OR words of the packed-record decision, fp_pipe_pk.h): the
// atomic only when this block adds a bit.  Most blocks find every bit set already, and atomics on one
// word serialise: config 4 issued 2 per scenario block from each of three kernels.
__device__ __forceinline__ void fp_or_new_bits(uint32_t *w, uint32_t bits) {
    if (bits & ~*(volatile uint32_t *)w) atomicOr(w, bits);
}

struct fp_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // kernel-side error words (a CSR index out of range, the pipeline's deadlock guard):
    // kernels atomicMax into the CURRENT word `d_err`.  fp_dev_* calls use the async word
    // (d_err_base[0]): sticky until fp_ctx_sync reports and clears it.  A host-pointer call
    // switches to its own word (d_err_base[HOST_ERR]) for its duration and reports only that
    // one, so an earlier async failure neither fails an unrelated synchronous call nor gets
    // cleared by it
    static constexpr uint32_t HOST_ERR = 32;
    uint32_t *d_err_base = nullptr;
    uint32_t *d_err = nullptr;
    // per-context options (fp_ctx_set_option; FP_OPT_AUTO = production default)
    int64_t opt[FP_OPT_COUNT];
    // recorded on the launch stream at the end of every fp_dev_* call: fp_ctx_set_stream
    // waits on it instead of synchronising a stream handle the caller may have destroyed
    hipEvent_t last_ev = nullptr;
    // device workspace: a bump arena reset at the start of every API call
    char *ws = nullptr;
    size_t ws_cap = 0, ws_top = 0;
    // host-API staging arena (device memory holding copies of host inputs)
    char *stage = nullptr;
    size_t stage_cap = 0, stage_top = 0;
    // pinned host bounce buffer for small read-backs
    uint64_t *h_small = nullptr;
    // pinned host staging of host-API results: copied to the caller only when every
    // kernel and every device-to-host copy succeeded (all-or-nothing)
    char *h_stage = nullptr;
    size_t h_stage_cap = 0;
    // pinned host staging of host-API inputs (one host-to-device copy per call); h_in_ev marks the
    // last copy out of it, waited on before the buffer is written again
    char *h_in = nullptr;
    size_t h_in_cap = 0;
    hipEvent_t h_in_ev = nullptr;
    // mapped pinned host memory of fp_plan_stage's one-launch path (fp_small.hip): the kernel reads
    // its inputs from and writes its results to it (h_map on the host, d_map on the device)
    char *h_map = nullptr;
    void *d_map = nullptr;
    size_t h_map_cap = 0;
    // fp_plan_stage's one-wave path for stages of <= 64 services (k_plan_tiny): its tagged result
    // words in mapped pinned host memory, and the tag of the last call (1..255)
    char *h_tiny = nullptr;
    void *d_tiny = nullptr;
    uint32_t tiny_tag = 0;
    // the asynchronous levelizer's work queues (fp_order.hip), kept between calls: a clean finish
    // leaves them empty, and the flag in their last 256 bytes tells the next call whether to refill
    void *lvl_q = nullptr;
    // the last placement's range words (CN_ORC.. of its workspace: OR cpu, OR mem, kernel path),
    // read by fp_ctx_place_path
    uint32_t *last_rng = nullptr;
    size_t lvl_q_cap = 0;
    // profiling
    bool profile = false;
    struct Rec { int kid; hipEvent_t a, b; };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    double total_ms[FP_K_COUNT] = {0};
    uint64_t launches[FP_K_COUNT] = {0};
};

// arena helpers (return nullptr on failure; callers map to FP_ENOMEM)
void fp_ws_reset(fp_ctx *c);
int fp_ws_reserve(fp_ctx *c, size_t bytes);  // ensure capacity (may sync + realloc)
void *fp_ws_take(fp_ctx *c, size_t bytes);   // 256-B aligned slice
void fp_stage_reset(fp_ctx *c);
int fp_stage_reserve(fp_ctx *c, size_t bytes);
void *fp_stage_take(fp_ctx *c, size_t bytes);

// profiling brackets around a launch on ctx->stream
void fp_prof_begin(fp_ctx *c, int kid, hipEvent_t *a);
void fp_prof_end(fp_ctx *c, int kid, hipEvent_t a);

// synchronise the stream, read the current kernel error word and clear it (0 or -FP_E*)
int fp_take_err(fp_ctx *c);
// the end of every fp_dev_* entry point (fp_ctx.hip): records c->last_ev on the context's stream,
// which fp_ctx_set_stream waits on before a switch; returns rc (FP_EDEVICE if the record failed)
int fp_dev_done(fp_ctx *c, int rc);

// option value, or `dflt` when the option is FP_OPT_AUTO
static inline int64_t fp_opt(const fp_ctx *c, int k, int64_t dflt) {
    return (c && c->opt[k] != FP_OPT_AUTO) ? c->opt[k] : dflt;
}

// a host-pointer call's own kernel error word for its duration (fp_internal.h fp_ctx)
// The word is cleared on entry (stream-ordered), so an error a previous host call's kernels
// raised after that call exited early (a HIP failure, ENOMEM mid-call) is not reported here.
// Built after hipSetDevice(c->device) (the clear is issued on the context's device); `rc` is the
// clear's result, which the caller returns when it failed.
struct fp_host_err_scope {
    fp_ctx *c;
    int rc;
    explicit fp_host_err_scope(fp_ctx *cc) : c(cc) {
        c->d_err = c->d_err_base + fp_ctx::HOST_ERR;
        const hipError_t e = hipMemsetAsync(c->d_err, 0, 4, c->stream);
        rc = e == hipSuccess ? FP_OK : fp_hip_fail(e);
    }
    ~fp_host_err_scope() { c->d_err = c->d_err_base; }
};

static inline uint32_t fp_bitwidth(uint64_t v) {
    uint32_t b = 0;
    while (v) { b++; v >>= 1; }
    return b;
}

// ---- entry points shared between translation units ----
int fp_dev_place_batch_impl(fp_ctx *c, const fp_batch *b);
int fp_dev_levelize_impl(fp_ctx *c, const fp_graph *g, uint32_t *level, uint32_t *order,
                         uint32_t *n_cycle_dev);
int fp_dev_legacy_order_impl(fp_ctx *c, const fp_graph *g, uint32_t *perm);
int fp_dev_feasibility_impl(fp_ctx *c, const fp_containers *cs, const fp_nodes *ns,
                            uint32_t *first, uint32_t *count, uint64_t *bitmap);
int fp_dev_feasibility_batch_impl(fp_ctx *c, const fp_batch *b, uint32_t *first, uint32_t *count);

// tile-pipeline FFD (fp_pipe.hip)
bool fp_pipe_plan(const fp_ctx *c, uint32_t S, uint32_t N, uint32_t *G_out, uint32_t *W_out, uint32_t *B_out,
                  size_t *lds_out);
int fp_place_geometry_impl(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, uint32_t *out);
size_t fp_pipe_ws_bytes(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N);
int fp_place_ws_bytes_impl(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, uint64_t *bytes);
// bucket thresholds of the candidate masks: K ascending values, T[0] = 0
constexpr int FP_BUCKETS = 32;
// geometric from lo to hi (host and device: fp_place.hip k_thresholds)
__host__ __device__ inline void fp_thresholds(uint32_t lo, uint32_t hi, uint32_t *T) {
    T[0] = 0;
    if (lo == 0) lo = 1;
    if (hi < lo) hi = lo;
    const double r = pow((double)hi / (double)lo, 1.0 / (double)(FP_BUCKETS - 2));
    double v = (double)lo;
    for (int k = 1; k < FP_BUCKETS; ++k) {
        uint32_t x = k == FP_BUCKETS - 1 ? hi : (uint32_t)ceil(v);
        if (x < T[k - 1]) x = T[k - 1];
        if (x > hi) x = hi;
        T[k] = x;
        v *= r;
    }
}
// the FFD-sorted SoA [S][C] the pipeline streams (fp_pipe.hip)
struct fp_pipe_soa {
    uint32_t *s_cpu, *s_mem, *s_req, *s_conf, *s_idx;
};
int fp_pipe_soa_take(fp_ctx *c, size_t SC, fp_pipe_soa *soa);
// 1 when the position word carries the bucket indices (bits 21-30)
uint32_t fp_pipe_kpack(const fp_ctx *c, uint32_t C);
// ready: the per-scenario LDS sort already wrote order, s_cpu, s_mem and s_idx (only the
// req / conf / CYCLE gather remains); null: gather everything from order + sorted keys.
// thr: the pipeline's bucket thresholds in device memory ([FP_BUCKETS] cpu, then mem)
// rng: [2] the OR of every container cpu / mem value of the batch (the sort kernels wrote it); the
// pipeline adds the nodes' and runs the packed kernel when the values pack (null: u32 kernels only)
int fp_pipe_launch(fp_ctx *c, uint32_t S, uint32_t C, uint32_t N, uint32_t scen_base, const uint32_t *order,
                   const void *skeys, uint32_t key_bytes, uint32_t mbits, uint64_t cmax, uint64_t mmax,
                   const uint32_t *cval, const uint32_t *mval, const fp_batch *b, const uint32_t *thr,
                   const fp_pipe_soa *ready, uint32_t *rng);

// ---- device helpers ----
namespace fpd {

constexpr uint64_t GAMMA = 0x9E3779B97F4A7C15ull;
constexpr uint64_t TAG_CONT = 0xC0C0C0C0C0C0C0C0ull;
constexpr uint64_t TAG_NODE = 0x5E5E5E5E5E5E5E5Eull;

// SPEC.md 3.1: draw(seed, k) = (k+1)-th SplitMix64 output from state `seed`.
__host__ __device__ inline uint64_t draw(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * GAMMA;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t scenario_seed(uint64_t seed, uint32_t s) {
    return seed ^ ((uint64_t)s * GAMMA);
}

// Single node-fit predicate (SPEC.md 2.3); sched handled by callers.
__device__ __forceinline__ bool fits(uint32_t cpu, uint32_t mem, uint32_t req, uint32_t conf,
                                     uint32_t cf, uint32_t mf, uint32_t lab, uint32_t cu) {
    return (cf >= cpu) & (mf >= mem) & ((lab & req) == req) & ((cu & conf) == 0u);
}

__device__ __forceinline__ uint64_t pack_cost(uint32_t rej, uint32_t used, uint32_t id) {
    uint64_t r = rej > 0xFFFFFFu ? 0xFFFFFFu : rej;
    uint64_t u = used > 0xFFFFFFu ? 0xFFFFFFu : used;
    return (r << 40) | (u << 16) | (uint64_t)(id & 0xFFFFu);
}

}  // namespace fpd
