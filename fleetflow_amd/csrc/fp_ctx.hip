// fp_ctx.hip -- context lifetime, device arenas, profiling and the synchronous
// host-pointer entry points of include/fleetplace.h.
//
// The host API copies caller arrays into a device staging arena, runs the same
// device pipeline as fp_dev_*, and copies results back only when every kernel
// succeeded ("no partial writes on error").
#include "fp_internal.h"
#include <string.h>
#include <stdlib.h>

int fp_hip_fail(hipError_t e) {
    (void)e;
    if (e == hipErrorOutOfMemory) return FP_ENOMEM;
    return FP_EDEVICE;
}

extern "C" const char *fp_strerror(int code) {
    switch (code) {
    case FP_OK: return "ok";
    case FP_EINVAL: return "invalid argument";
    case FP_ENOMEM: return "out of memory";
    case FP_EDEVICE: return "no gfx950 device or HIP runtime error";
    case FP_EOVERFLOW: return "count overflow";
    case FP_ECORRUPT: return "input violates an invariant";
    default: return "unknown error";
    }
}

extern "C" int fp_abi_version(void) { return FP_ABI_VERSION; }

extern "C" int fp_ctx_create(fp_ctx **out, int device) {
    if (!out) return FP_EINVAL;
    *out = nullptr;
    if (device < 0) return FP_EINVAL;  // no CPU backend by design
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device >= n) return FP_EDEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return FP_EDEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FP_EDEVICE;
    fp_ctx *c = new fp_ctx();
    c->device = device;
    for (int k = 0; k < FP_OPT_COUNT; ++k) c->opt[k] = FP_OPT_AUTO;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_err_base, 256) != hipSuccess ||
        hipEventCreateWithFlags(&c->last_ev, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(&c->h_small, 4096, hipHostMallocDefault) != hipSuccess) {
        fp_ctx_destroy(c);
        return FP_EDEVICE;
    }
    if (hipMemset(c->d_err_base, 0, 256) != hipSuccess) {
        fp_ctx_destroy(c);
        return FP_EDEVICE;
    }
    c->d_err = c->d_err_base;
    c->stream = c->own_stream;
    *out = c;
    return FP_OK;
}

extern "C" void fp_ctx_destroy(fp_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->last_ev) (void)hipEventSynchronize(c->last_ev);
    for (auto &r : c->pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    if (c->ws) (void)hipFree(c->ws);
    if (c->stage) (void)hipFree(c->stage);
    if (c->d_err_base) (void)hipFree(c->d_err_base);
    if (c->last_ev) (void)hipEventDestroy(c->last_ev);
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->h_in_ev) (void)hipEventSynchronize(c->h_in_ev);
    if (c->h_in) (void)hipHostFree(c->h_in);
    if (c->h_in_ev) (void)hipEventDestroy(c->h_in_ev);
    if (c->h_map) (void)hipHostFree(c->h_map);
    if (c->h_tiny) (void)hipHostFree(c->h_tiny);
    if (c->lvl_q) (void)hipFree(c->lvl_q);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

// Switching streams first waits for this context's work on the old one: the workspace arena
// is reset by every call, so it must not overlap a call on the new stream.  It waits on the
// event the last fp_dev_* call recorded, never on the old stream handle itself, which the
// caller may already have destroyed.
extern "C" int fp_ctx_set_stream(fp_ctx *c, void *s) {
    if (!c) return FP_EINVAL;
    if ((hipStream_t)s != c->stream) {
        FP_HIP(hipSetDevice(c->device));
        FP_HIP(hipEventSynchronize(c->last_ev));
    }
    c->stream = (hipStream_t)s;  // NULL = HIP null stream
    return FP_OK;
}

extern "C" int fp_ctx_set_option(fp_ctx *c, int k, int64_t v) {
    if (!c || k < 0 || k >= FP_OPT_COUNT || v < FP_OPT_AUTO) return FP_EINVAL;
    c->opt[k] = v;
    return FP_OK;
}

extern "C" int fp_ctx_get_option(fp_ctx *c, int k, int64_t *v) {
    if (!c || !v || k < 0 || k >= FP_OPT_COUNT) return FP_EINVAL;
    *v = c->opt[k];
    return FP_OK;
}

extern "C" int fp_ctx_reset_stream(fp_ctx *c) {
    return fp_ctx_set_stream(c, c ? (void *)c->own_stream : nullptr);
}

// Waits for every fp_dev_* call queued on the context's stream and reports the first
// kernel-side error any of them raised since the last report (then clears it).
extern "C" int fp_ctx_sync(fp_ctx *c) {
    if (!c) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    c->d_err = c->d_err_base;
    return fp_take_err(c);
}

// the end of every fp_dev_* entry point: remember where this context's work ends
int fp_dev_done(fp_ctx *c, int rc) {
    if (hipEventRecord(c->last_ev, c->stream) != hipSuccess && rc == FP_OK) rc = FP_EDEVICE;
    return rc;
}

// ---- arenas ----------------------------------------------------------------
static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

void fp_ws_reset(fp_ctx *c) { c->ws_top = 0; }
int fp_ws_reserve(fp_ctx *c, size_t bytes) {
    if (bytes <= c->ws_cap) return FP_OK;
    FP_HIP(hipStreamSynchronize(c->stream));
    if (c->ws) (void)hipFree(c->ws);
    c->ws = nullptr;
    c->ws_cap = 0;
    size_t cap = align256(bytes + bytes / 4 + 4096);
    FP_HIP(hipMalloc(&c->ws, cap));
    c->ws_cap = cap;
    return FP_OK;
}
void *fp_ws_take(fp_ctx *c, size_t bytes) {
    size_t top = align256(c->ws_top);
    if (top + bytes > c->ws_cap) return nullptr;
    c->ws_top = top + bytes;
    return c->ws + top;
}
void fp_stage_reset(fp_ctx *c) { c->stage_top = 0; }
int fp_stage_reserve(fp_ctx *c, size_t bytes) {
    if (bytes <= c->stage_cap) return FP_OK;
    FP_HIP(hipStreamSynchronize(c->stream));
    if (c->stage) (void)hipFree(c->stage);
    c->stage = nullptr;
    c->stage_cap = 0;
    size_t cap = align256(bytes + bytes / 4 + 4096);
    FP_HIP(hipMalloc(&c->stage, cap));
    c->stage_cap = cap;
    return FP_OK;
}
void *fp_stage_take(fp_ctx *c, size_t bytes) {
    size_t top = align256(c->stage_top);
    if (top + bytes > c->stage_cap) return nullptr;
    c->stage_top = top + bytes;
    return c->stage + top;
}

int fp_take_err(fp_ctx *c) {
    FP_HIP(hipMemcpyAsync(c->h_small, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    FP_HIP(hipStreamSynchronize(c->stream));
    const uint32_t e = ((const uint32_t *)c->h_small)[0];
    if (!e) return FP_OK;
    FP_HIP(hipMemsetAsync(c->d_err, 0, 4, c->stream));
    FP_HIP(hipStreamSynchronize(c->stream));
    return -(int)e;
}

// ---- profiling ---------------------------------------------------------------
static hipEvent_t ev_get(fp_ctx *c) {
    if (!c->pool.empty()) {
        hipEvent_t e = c->pool.back();
        c->pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}
void fp_prof_begin(fp_ctx *c, int kid, hipEvent_t *a) {
    (void)kid;
    *a = nullptr;
    if (!c->profile) return;
    *a = ev_get(c);
    (void)hipEventRecord(*a, c->stream);
}
void fp_prof_end(fp_ctx *c, int kid, hipEvent_t a) {
    if (!c->profile || !a) return;
    hipEvent_t b = ev_get(c);
    (void)hipEventRecord(b, c->stream);
    c->pending.push_back({kid, a, b});
}
extern "C" int fp_ctx_profile(fp_ctx *c, int enable) {
    if (!c) return FP_EINVAL;
    c->profile = enable != 0;
    for (int k = 0; k < FP_K_COUNT; ++k) { c->total_ms[k] = 0; c->launches[k] = 0; }
    return FP_OK;
}
extern "C" int fp_ctx_kernel_stats(fp_ctx *c, int kid, double *total_ms, uint64_t *launches) {
    if (!c || kid < 0 || kid >= FP_K_COUNT) return FP_EINVAL;
    for (auto &r : c->pending) {
        float ms = 0.f;
        FP_HIP(hipEventSynchronize(r.b));
        FP_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        c->total_ms[r.kid] += ms;
        c->launches[r.kid] += 1;
        c->pool.push_back(r.a);
        c->pool.push_back(r.b);
    }
    c->pending.clear();
    if (total_ms) *total_ms = c->total_ms[kid];
    if (launches) *launches = c->launches[kid];
    return FP_OK;
}

// ---- device-pointer entry points ----------------------------------------------
extern "C" int fp_dev_place_batch(fp_ctx *c, const fp_batch *b) {
    if (!c || !b) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_dev_done(c, fp_dev_place_batch_impl(c, b));
}
extern "C" int fp_dev_levelize(fp_ctx *c, const fp_graph *g, uint32_t *level, uint32_t *order,
                               uint32_t *n_cycle_dev) {
    if (!c || !g) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_dev_done(c, fp_dev_levelize_impl(c, g, level, order, n_cycle_dev));
}
extern "C" int fp_dev_legacy_order(fp_ctx *c, const fp_graph *g, uint32_t *perm) {
    if (!c || !g) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_dev_done(c, fp_dev_legacy_order_impl(c, g, perm));
}
extern "C" int fp_place_ws_bytes(fp_ctx *c, uint32_t n_scen, uint32_t n_containers, uint32_t n_nodes,
                                 uint64_t *bytes_out) {
    if (!c || !bytes_out) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_place_ws_bytes_impl(c, n_scen, n_containers, n_nodes, bytes_out);
}
extern "C" int fp_place_geometry(fp_ctx *c, uint32_t n_scen, uint32_t n_containers, uint32_t n_nodes,
                                 uint32_t *out) {
    if (!c || !out) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_place_geometry_impl(c, n_scen, n_containers, n_nodes, out);
}
extern "C" int fp_dev_feasibility_batch(fp_ctx *c, const fp_batch *b, uint32_t *first, uint32_t *count) {
    if (!c || !b) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_dev_done(c, fp_dev_feasibility_batch_impl(c, b, first, count));
}
extern "C" int fp_dev_feasibility(fp_ctx *c, const fp_containers *cs, const fp_nodes *ns,
                                  uint32_t *first, uint32_t *count, uint64_t *bitmap) {
    if (!c || !cs || !ns) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    return fp_dev_done(c, fp_dev_feasibility_impl(c, cs, ns, first, count, bitmap));
}

// ---- host-pointer entry points -------------------------------------------------
template <class T>
static T *stage_in(fp_ctx *c, const T *h, size_t n, int *rc) {
    if (*rc) return nullptr;
    if (!h) return nullptr;
    T *d = (T *)fp_stage_take(c, n * sizeof(T) + 4);
    if (!d) { *rc = FP_ENOMEM; return nullptr; }
    if (n && hipMemcpyAsync(d, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream) != hipSuccess)
        *rc = FP_EDEVICE;
    return d;
}
template <class T>
static T *stage_out(fp_ctx *c, size_t n, int *rc) {
    if (*rc) return nullptr;
    T *d = (T *)fp_stage_take(c, n * sizeof(T) + 4);
    if (!d) *rc = FP_ENOMEM;
    return d;
}
// Results of a host-pointer call: every device buffer goes to pinned staging first; the
// caller's buffers are written only after the kernels' error word and every copy came
// back clean ("on error nothing is written", fleetplace.h).
struct OutCopy {
    void *h;
    const void *d;
    size_t bytes;
};
static int copy_back_all(fp_ctx *c, const OutCopy *o, int n) {
    size_t total = 0;
    for (int i = 0; i < n; ++i)
        if (o[i].h && o[i].bytes) total += align256(o[i].bytes);
    if (total > c->h_stage_cap) {
        if (c->h_stage) (void)hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_cap = 0;
        const size_t cap = align256(total + total / 4 + 4096);
        FP_HIP(hipHostMalloc(&c->h_stage, cap, hipHostMallocDefault));
        c->h_stage_cap = cap;
    }
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
        if (!o[i].h || !o[i].bytes) continue;
        FP_HIP(hipMemcpyAsync(c->h_stage + off, o[i].d, o[i].bytes, hipMemcpyDeviceToHost, c->stream));
        off += align256(o[i].bytes);
    }
    const int rc = fp_take_err(c);  // synchronises the copies too
    if (rc) return rc;
    off = 0;
    for (int i = 0; i < n; ++i) {
        if (!o[i].h || !o[i].bytes) continue;
        memcpy(o[i].h, c->h_stage + off, o[i].bytes);
        off += align256(o[i].bytes);
    }
    return FP_OK;
}

// Small host-pointer calls (a fleet.kdl stage: config 1) pay per HIP call, not per byte: the
// inputs go through one pinned buffer and ONE host-to-device copy, and the results plus the
// call's error word come back in ONE device-to-host copy of the contiguous staging span
// (6 HIP calls per fp_levelize instead of 10; the results are still written only when the error
// word is clean).
struct InCopy {
    const void *h;
    size_t bytes;
    const void **d;  // receives the device copy (nullptr when h is null)
};
static int stage_in_packed(fp_ctx *c, const InCopy *in, int n) {
    size_t total = 0;
    for (int i = 0; i < n; ++i)
        if (in[i].h) total += align256(in[i].bytes + 4);
    if (!total) {
        for (int i = 0; i < n; ++i) *in[i].d = nullptr;
        return FP_OK;
    }
    if (c->h_in_ev) FP_HIP(hipEventSynchronize(c->h_in_ev));  // the previous copy out of h_in is done
    if (total > c->h_in_cap) {
        if (c->h_in) (void)hipHostFree(c->h_in);
        c->h_in = nullptr;
        c->h_in_cap = 0;
        const size_t cap = align256(total + total / 4 + 4096);
        FP_HIP(hipHostMalloc(&c->h_in, cap, hipHostMallocDefault));
        c->h_in_cap = cap;
    }
    if (!c->h_in_ev) FP_HIP(hipEventCreateWithFlags(&c->h_in_ev, hipEventDisableTiming));
    char *d = (char *)fp_stage_take(c, total);
    if (!d) return FP_ENOMEM;
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
        if (!in[i].h) { *in[i].d = nullptr; continue; }
        memcpy(c->h_in + off, in[i].h, in[i].bytes);
        *in[i].d = d + off;
        off += align256(in[i].bytes + 4);
    }
    FP_HIP(hipMemcpyAsync(d, c->h_in, total, hipMemcpyHostToDevice, c->stream));
    FP_HIP(hipEventRecord(c->h_in_ev, c->stream));
    return FP_OK;
}
// Results from stage_out buffers taken one after another (a contiguous span of the staging
// arena): the call's error word is copied behind them on the device, the span comes back in one
// copy, and the caller's buffers are written only when that word is clean.
static int copy_back_span(fp_ctx *c, const OutCopy *o, int n) {
    const char *lo = nullptr, *hi = nullptr;
    for (int i = 0; i < n; ++i) {
        if (!o[i].d) continue;
        const char *a = (const char *)o[i].d, *b = a + o[i].bytes;
        if (!lo || a < lo) lo = a;
        if (!hi || b > hi) hi = b;
    }
    uint32_t *slot = (uint32_t *)fp_stage_take(c, 4);
    if (!slot) return FP_ENOMEM;
    if (!lo) lo = (const char *)slot;
    if ((const char *)slot < hi) return FP_EINVAL;  // not the layout this helper assumes
    const size_t span = (size_t)((const char *)slot + 4 - lo);
    if (span > c->h_stage_cap) {
        if (c->h_stage) (void)hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_cap = 0;
        const size_t cap = align256(span + span / 4 + 4096);
        FP_HIP(hipHostMalloc(&c->h_stage, cap, hipHostMallocDefault));
        c->h_stage_cap = cap;
    }
    FP_HIP(hipMemcpyAsync(slot, c->d_err, 4, hipMemcpyDeviceToDevice, c->stream));
    FP_HIP(hipMemcpyAsync(c->h_stage, lo, span, hipMemcpyDeviceToHost, c->stream));
    FP_HIP(hipStreamSynchronize(c->stream));
    const uint32_t e = *(const uint32_t *)(c->h_stage + ((const char *)slot - lo));
    if (e) {
        FP_HIP(hipMemsetAsync(c->d_err, 0, 4, c->stream));
        FP_HIP(hipStreamSynchronize(c->stream));
        return -(int)e;
    }
    for (int i = 0; i < n; ++i)
        if (o[i].h && o[i].bytes) memcpy(o[i].h, c->h_stage + ((const char *)o[i].d - lo), o[i].bytes);
    return FP_OK;
}

extern "C" int fp_legacy_order(fp_ctx *c, const fp_graph *g, uint32_t *perm_out) {
    if (!c || !g || (g->n_vertices && (!g->has_deps || !perm_out))) return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    fp_host_err_scope es(c);
    if (es.rc) return es.rc;
    const size_t V = g->n_vertices;
    int rc = fp_stage_reserve(c, 2 * V * 4 + 8192);
    if (rc) return rc;
    fp_stage_reset(c);
    fp_graph dg = *g;
    const void *dhd = nullptr;
    const InCopy in[] = {{g->has_deps, V, &dhd}};
    if ((rc = stage_in_packed(c, in, 1))) return rc;
    dg.has_deps = (const uint8_t *)dhd;
    dg.row_ptr = nullptr;
    dg.col = nullptr;
    uint32_t *dperm = stage_out<uint32_t>(c, V, &rc);
    if (rc) return rc;
    rc = fp_dev_legacy_order_impl(c, &dg, dperm);
    if (rc) return rc;
    const OutCopy o[] = {{perm_out, dperm, V * 4}};
    return copy_back_span(c, o, 1);
}

extern "C" int fp_levelize(fp_ctx *c, const fp_graph *g, uint32_t *level_out, uint32_t *order_out,
                           uint32_t *n_cycle_out) {
    if (!c || !g) return FP_EINVAL;
    const size_t V = g->n_vertices, E = g->n_edges;
    if (V && (!g->has_deps || !g->row_ptr || !level_out || !order_out)) return FP_EINVAL;
    if (E && !g->col) return FP_EINVAL;
    if (V == 0) {
        if (E) return FP_ECORRUPT;
        if (n_cycle_out) *n_cycle_out = 0;
        return FP_OK;
    }
    // the CSR is validated on the device (k_check_csr, k_indeg): FP_ECORRUPT
    FP_HIP(hipSetDevice(c->device));
    fp_host_err_scope es(c);
    if (es.rc) return es.rc;
    int rc = fp_stage_reserve(c, (V + 1) * 4 + E * 4 + V + 2 * V * 4 + 16 * 256);
    if (rc) return rc;
    fp_stage_reset(c);
    fp_graph dg = *g;
    const void *drp = nullptr, *dcol = nullptr, *dhd = nullptr;
    const InCopy in[] = {{g->row_ptr, (V + 1) * 4, &drp}, {E ? g->col : nullptr, E * 4, &dcol},
                         {g->has_deps, V, &dhd}};
    if ((rc = stage_in_packed(c, in, 3))) return rc;
    dg.row_ptr = (const uint32_t *)drp;
    dg.col = (const uint32_t *)dcol;
    dg.has_deps = (const uint8_t *)dhd;
    uint32_t *dlev = stage_out<uint32_t>(c, V, &rc);
    uint32_t *dord = stage_out<uint32_t>(c, V, &rc);
    uint32_t *dcyc = stage_out<uint32_t>(c, 1, &rc);
    if (rc) return rc;
    rc = fp_dev_levelize_impl(c, &dg, dlev, dord, dcyc);
    if (rc) return rc;
    const OutCopy o[] = {{level_out, dlev, V * 4}, {order_out, dord, V * 4}, {n_cycle_out, dcyc, 4}};
    return copy_back_span(c, o, 3);
}

static int batch_host(fp_ctx *c, const fp_batch *b) {
    const size_t S = b->n_scen, C = b->n_containers, N = b->n_nodes;
    const size_t SC = S * C, SN = S * N;
    if (S && C && (!b->cpu_m || !b->mem_mib || !b->req_labels || !b->conflict || !b->assign ||
                   !b->reason))
        return FP_EINVAL;
    if (S && N && (!b->cpu_free || !b->mem_free || !b->labels || !b->conflict_used ||
                   !b->schedulable))
        return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    fp_host_err_scope es(c);
    if (es.rc) return es.rc;
    int rc = fp_stage_reserve(c, SC * (4 * 6 + 1) + SN * (4 * 4 + 1) + S * 8 + 16 * 256);
    if (rc) return rc;
    fp_stage_reset(c);
    fp_batch d = *b;
    d.cpu_m = stage_in(c, b->cpu_m, SC, &rc);
    d.mem_mib = stage_in(c, b->mem_mib, SC, &rc);
    d.req_labels = stage_in(c, b->req_labels, SC, &rc);
    d.conflict = stage_in(c, b->conflict, SC, &rc);
    d.level = b->level ? stage_in(c, b->level, SC, &rc) : nullptr;
    d.cpu_free = stage_in(c, b->cpu_free, SN, &rc);
    d.mem_free = stage_in(c, b->mem_free, SN, &rc);
    d.labels = stage_in(c, b->labels, SN, &rc);
    d.conflict_used = stage_in(c, b->conflict_used, SN, &rc);
    d.schedulable = stage_in(c, b->schedulable, SN, &rc);
    d.assign = stage_out<uint32_t>(c, SC, &rc);
    d.reason = stage_out<uint8_t>(c, SC, &rc);
    d.cost = stage_out<uint64_t>(c, S, &rc);
    if (rc) return rc;
    rc = fp_dev_place_batch_impl(c, &d);
    if (rc) return rc;
    const OutCopy o[] = {{b->assign, d.assign, SC * 4},          {b->reason, d.reason, SC},
                         {b->cost, d.cost, S * 8},                {b->cpu_free, d.cpu_free, SN * 4},
                         {b->mem_free, d.mem_free, SN * 4},       {b->conflict_used, d.conflict_used, SN * 4}};
    return copy_back_all(c, o, 6);
}

extern "C" int fp_place_batch(fp_ctx *c, const fp_batch *b) {
    if (!c || !b) return FP_EINVAL;
    return batch_host(c, b);
}

extern "C" int fp_place(fp_ctx *c, const fp_containers *cs, fp_nodes *ns, const uint32_t *level,
                        uint32_t *assign_out, uint8_t *reason_out) {
    if (!c || !cs || !ns) return FP_EINVAL;
    fp_batch b;
    memset(&b, 0, sizeof(b));
    b.n_scen = 1;
    b.scen_base = 0;
    b.n_containers = cs->n;
    b.n_nodes = ns->n;
    b.cpu_m = cs->cpu_m;
    b.mem_mib = cs->mem_mib;
    b.req_labels = cs->req_labels;
    b.conflict = cs->conflict;
    b.level = level;
    b.cpu_free = ns->cpu_free;
    b.mem_free = ns->mem_free;
    b.labels = ns->labels;
    b.conflict_used = ns->conflict_used;
    b.schedulable = ns->schedulable;
    b.assign = assign_out;
    b.reason = reason_out;
    b.cost = nullptr;
    return batch_host(c, &b);
}

extern "C" int fp_feasibility(fp_ctx *c, const fp_containers *cs, const fp_nodes *ns,
                              uint32_t *first_out, uint32_t *count_out, uint64_t *bitmap_out) {
    if (!c || !cs || !ns) return FP_EINVAL;
    const size_t C = cs->n, N = ns->n, WC = (C + 63) / 64;
    if (C && (!cs->cpu_m || !cs->mem_mib || !cs->req_labels || !cs->conflict || !first_out ||
              !count_out))
        return FP_EINVAL;
    if (N && (!ns->cpu_free || !ns->mem_free || !ns->labels || !ns->conflict_used ||
              !ns->schedulable))
        return FP_EINVAL;
    FP_HIP(hipSetDevice(c->device));
    fp_host_err_scope es(c);
    if (es.rc) return es.rc;
    int rc = fp_stage_reserve(c, C * 24 + N * 17 + (bitmap_out ? WC * N * 8 : 0) + 16 * 256);
    if (rc) return rc;
    fp_stage_reset(c);
    fp_containers dc = *cs;
    fp_nodes dn = *ns;
    dc.cpu_m = stage_in(c, cs->cpu_m, C, &rc);
    dc.mem_mib = stage_in(c, cs->mem_mib, C, &rc);
    dc.req_labels = stage_in(c, cs->req_labels, C, &rc);
    dc.conflict = stage_in(c, cs->conflict, C, &rc);
    dn.cpu_free = stage_in(c, ns->cpu_free, N, &rc);
    dn.mem_free = stage_in(c, ns->mem_free, N, &rc);
    dn.labels = stage_in(c, ns->labels, N, &rc);
    dn.conflict_used = stage_in(c, ns->conflict_used, N, &rc);
    dn.schedulable = stage_in(c, ns->schedulable, N, &rc);
    uint32_t *dfirst = stage_out<uint32_t>(c, C, &rc);
    uint32_t *dcount = stage_out<uint32_t>(c, C, &rc);
    uint64_t *dbits = bitmap_out ? stage_out<uint64_t>(c, WC * N, &rc) : nullptr;
    if (rc) return rc;
    rc = fp_dev_feasibility_impl(c, &dc, &dn, dfirst, dcount, dbits);
    if (rc) return rc;
    const OutCopy o[] = {{first_out, dfirst, C * 4}, {count_out, dcount, C * 4}, {bitmap_out, dbits, WC * N * 8}};
    return copy_back_all(c, o, 3);
}
