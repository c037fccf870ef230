/*
 * fleetplace.h -- C ABI of the MI355X-native FleetFlow placement planner
 * (libfleetplace.so, HIP/gfx950).  This is the drop-in boundary for the
 * reference's plan path.
 *
 * Reference interfaces this ABI replaces (paths relative to chronista-club/fleetflow):
 *   fp_legacy_order   <- fn order_by_dependencies(&[String], &Flow) -> Vec<String>
 *                        crates/fleetflow-container/src/engine.rs:64-85
 *                        (names -> u32 ids in stage order are mapped by the caller;
 *                         strings never cross this ABI)
 *   fp_levelize       <- new: Kahn start levels generalising engine.rs:67-85
 *                        (replaces the call at engine.rs:157 when levels are wanted)
 *   fp_place          <- `stages[stage].servers.first()` with "local" fallback
 *                        crates/fleetflow-controlplane/src/handlers/deploy.rs:386-398
 *                        (N = 1, unconstrained capacity reproduces it exactly)
 *   fp_place_batch    <- new: what-if scenarios, one plan per scenario + packed cost
 *   fp_feasibility    <- new: stage-2 containers x nodes feasibility/score sweep
 *   fp_dev_feasibility_batch <- new: the same sweep over many what-if scenarios
 *
 * Conventions
 *   - All buffers are caller-owned; no allocation crosses the ABI.
 *   - fp_* take HOST pointers and are synchronous: on error nothing is written.
 *   - fp_dev_* take DEVICE (HBM) pointers of the context's device and are
 *     asynchronous on the context's stream.  Kernel-side errors of fp_dev_* calls
 *     (FP_ECORRUPT input, FP_EDEVICE from the placement pipeline's deadlock guard) are
 *     sticky: the first one raised is kept until fp_ctx_sync() reports it and clears it.
 *     A host-pointer call reports only the errors of its own kernels (it has its own error
 *     word): a pending asynchronous error neither fails it nor is cleared by it.
 *     fp_dev_* calls read nothing back: every data-dependent choice (key range, sort path,
 *     bucket thresholds, level count, a corrupt CSR) is made on the device, so a caller can
 *     queue call i+1 behind call i's collectives without a host stall.  The exceptions: the
 *     first call of a shape larger than any before it grows the context's workspace (one
 *     stream synchronisation), and FP_OPT_LEVELIZE_SYNC = 1 (the level-synchronous
 *     levelizer) reads its frontier size back once per 64 levels.
 *   - fp_ctx_set_stream first waits for the context's last fp_dev_* call (an event
 *     recorded on the old stream; the workspace is reused by every call).  It never
 *     touches the old stream handle itself, so a caller may destroy that stream once
 *     its own work on it is done.
 *   - The placement pipeline's bounded links (fp_place_geometry FP_GEOM_BOUNDED) need the
 *     launch's segments co-resident.  Bounded launches of one process are serialised per
 *     device inside the library (each waits on its own stream for the previous one), so
 *     contexts on several host threads may plan at once; other launches only delay them.
 *     Only work of OTHER processes that holds the device's slots indefinitely can still
 *     end a bounded launch in FP_EDEVICE after the deadlock guard (60 s), never in a
 *     wrong plan.
 *   - Return 0 (FP_OK) or a negative FP_E* code.  There is no CPU fallback:
 *     fp_ctx_create fails with FP_EDEVICE when no MI355X (gfx950) is present.
 *   - One fp_ctx per host thread; contexts are not shared.
 *   - Integer semantics only; results are bit-exact with the CPU oracle
 *     (oracle/fp_oracle.c) by construction.  Semantics: SPEC.md.
 */
#ifndef FLEETPLACE_H
#define FLEETPLACE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FP_ABI_VERSION 1

#define FP_OK 0
#define FP_EINVAL (-1)     /* bad argument / inconsistent sizes                  */
#define FP_ENOMEM (-2)     /* device or host allocation failed                   */
#define FP_EDEVICE (-3)    /* no gfx950 device, or a HIP runtime error           */
#define FP_EOVERFLOW (-4)  /* a count exceeds uint32 / a packed-cost field       */
#define FP_ECORRUPT (-5)   /* input violates an invariant (e.g. CSR col >= V)    */

#define FP_NONE 0xFFFFFFFFu /* "no node" / "no level" (cycle)                    */

enum fp_reason { FP_REASON_OK = 0, FP_REASON_NOFIT = 1, FP_REASON_CYCLE = 2 };

typedef struct fp_ctx fp_ctx;

/* depends_on graph as a REVERSED CSR: row d lists the vertices that depend on d.
 * has_deps[v] = 1 iff v is known in flow.services and its depends_on is non-empty
 * (the engine.rs:71-80 predicate). */
typedef struct {
    uint32_t n_vertices, n_edges;
    const uint32_t *row_ptr;  /* [n_vertices + 1] */
    const uint32_t *col;      /* [n_edges]        */
    const uint8_t *has_deps;  /* [n_vertices]     */
} fp_graph;

/* Container requests, SoA: integer CPU millicores, memory MiB, required label
 * bits, conflict bits (host-port bits | anti-affinity group bits). */
typedef struct {
    uint32_t n;
    const uint32_t *cpu_m, *mem_mib, *req_labels, *conflict;
} fp_containers;

/* Node table, SoA, in node-index order (stage.servers order for KDL input,
 * ORDER BY slug for the controlplane registry, db.rs:741-750).  cpu_free,
 * mem_free and conflict_used are updated in place by placement. */
typedef struct {
    uint32_t n;
    uint32_t *cpu_free, *mem_free;
    const uint32_t *labels;
    uint32_t *conflict_used;
    const uint8_t *schedulable; /* 0 = cordon/drain (model.rs:435-442) */
} fp_nodes;

/* S independent what-if scenarios, each C containers on its own N nodes.
 * Every array is scenario-major: container arrays [S][C], node arrays [S][N].
 * scen_base + n_scen <= 65536 (the packed cost keeps a 16-bit scenario id), else
 * FP_EOVERFLOW. */
typedef struct {
    uint32_t n_scen, scen_base;   /* scen_base: global id of scenario 0 (cost field) */
    uint32_t n_containers, n_nodes;
    const uint32_t *cpu_m, *mem_mib, *req_labels, *conflict;
    const uint32_t *level;        /* [S][C] or NULL: FP_NONE => CYCLE, not placed   */
    uint32_t *cpu_free, *mem_free;
    const uint32_t *labels;
    uint32_t *conflict_used;
    const uint8_t *schedulable;
    uint32_t *assign;             /* [S][C] node index or FP_NONE                   */
    uint8_t *reason;              /* [S][C] enum fp_reason                          */
    uint64_t *cost;               /* [S] (n_rejected:24 | n_nodes_used:24 | id:16)  */
} fp_batch;

/* ---- context ------------------------------------------------------------ */
int fp_ctx_create(fp_ctx **out, int device);
void fp_ctx_destroy(fp_ctx *ctx);
/* Launch on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream).
 * NULL selects the HIP null (default) stream; fp_ctx_reset_stream restores the
 * context's own non-blocking stream. */
int fp_ctx_set_stream(fp_ctx *ctx, void *hip_stream);
int fp_ctx_reset_stream(fp_ctx *ctx);
int fp_ctx_sync(fp_ctx *ctx);
const char *fp_strerror(int code);
int fp_abi_version(void);
/* Kernel timing (HIP events on the launch stream) for the roofline report.
 * kernel ids: see FP_K_* below. */
enum { FP_K_PLACE = 0, FP_K_SORT = 1, FP_K_FEAS = 2, FP_K_LEVEL = 3, FP_K_GEN = 4, FP_K_COUNT = 5 };
int fp_ctx_profile(fp_ctx *ctx, int enable);
int fp_ctx_kernel_stats(fp_ctx *ctx, int kernel_id, double *total_ms, uint64_t *launches);
/* The FFD kernel the last placement call on this context ran (waits for the stream): out[0] / out[1]
 * = the OR of every cpu / mem value of its batch (containers and schedulable nodes), out[2] = 1 for
 * the u32 records, 2 for the packed (cpu, mem) records (FP_OPT_PACKED), 0 if nothing ran. */
int fp_ctx_place_path(fp_ctx *ctx, uint32_t *out3);

/* Per-context tuning / test options.  FP_OPT_AUTO (-1) = the production choice (the
 * default of every option).  Nothing is read from the environment: an option changes
 * only the context it is set on.  The pipeline geometry options are hints a shape may
 * not be able to serve (the planner then falls back to the nearest valid geometry);
 * fp_place_geometry reports what a call will run.  Results are bit-exact whatever the
 * options (only the work schedule changes); FP_OPT_SPIN_TICKS, and FP_OPT_LINK_BOUNDED = 1
 * on a batch whose segments are not all resident, can make a call fail with FP_EDEVICE
 * (never a wrong plan). */
#define FP_OPT_AUTO (-1)
enum fp_option {
    FP_OPT_PIPE_W = 0,        /* stages (waves) per segment, >= 1                         */
    FP_OPT_PIPE_SEG = 1,      /* 64-node groups per segment, 1..40                         */
    FP_OPT_PIPE_R = 2,        /* LDS ring depth between stages, 2..6                        */
    FP_OPT_PIPE_LAG = 3,      /* segment ticket lag (0 = segments side by side)            */
    FP_OPT_LINK_SLOTS = 4,    /* bounded global link ring slots, >= 8                       */
    FP_OPT_LINK_BOUNDED = 5,  /* 0 = links hold every container, 1 = bounded rings          */
    FP_OPT_PIPE_FLUSH = 6,    /* idle-flush mask: bit 0 LDS rings, bit 1 global links      */
    FP_OPT_SPIN_TICKS = 7,    /* deadlock guard in 100 MHz ticks (auto: 60 s)               */
    FP_OPT_KPACK = 8,         /* 0 = bucket search per stage instead of packed buckets      */
    FP_OPT_SCEN_SORT = 9,     /* 0 = radix-key FFD order instead of the per-scenario LDS sort */
    FP_OPT_SEGSORT = 10,      /* ignored (kept for ABI stability): the radix path is always   */
                              /* segmented for S > 1 and device-wide for S == 1             */
    FP_OPT_SYSTOLIC = 11,     /* systolic group fill for queues of >= value containers (0 = off) */
    FP_OPT_LEVELIZE_SYNC = 12,/* 1 = level-synchronous Kahn instead of the async levelizer */
    FP_OPT_SYSTOLIC_EXTRA = 13, /* systolic steps past the queue length before the serial finish */
    FP_OPT_SCREEN = 14,       /* 0 = no stage-2 early-NOFIT screen: every container enters    */
    FP_OPT_PAYLOAD_LDS = 15,  /* 0 = random-gather payload instead of the LDS-chunked one      */
    FP_OPT_SYSTOLIC_VALU = 16,/* systolic step loop: 0 exec-masked, 1 VALU-only, auto/2 DPP-folded */
    FP_OPT_LINK_PUBLISH = 17, /* full slots per head publish on unbounded global links (auto 32) */
    FP_OPT_LEVEL_SORT = 18,   /* levelizer start order: 0 = radix sort, auto = LSD counting sort   */
    FP_OPT_LEVEL_SMALL = 19,  /* 0 = no one-launch levelizer (<= 512 vertices) / legacy order (<= 1024);
                                 2 = fp_plan_stage without its one-wave path (<= 64 services)   */
    FP_OPT_PIPE_PRIO = 20,    /* FFD wave priority: 0 off, 1 raised in the group loop, 2 for a batch's work */
    FP_OPT_INDEG_BIN = 21,    /* 0 = levelizer in-degrees by global atomics instead of binned in LDS */
    FP_OPT_PACKED = 22,       /* 0 = FFD on u32 records only; auto = packed (cpu, mem) records when the
                                 batch's values fit them (decided on the device, fp_pipe_pk.h)  */
    FP_OPT_COUNT = 23
};
int fp_ctx_set_option(fp_ctx *ctx, int option, int64_t value);
int fp_ctx_get_option(fp_ctx *ctx, int option, int64_t *value);

/* ---- host-pointer API (drop-in, synchronous) ---------------------------- */
/* A1 engine.rs:67-85: perm_out = stable partition (has_deps == 0 first). */
int fp_legacy_order(fp_ctx *ctx, const fp_graph *g, uint32_t *perm_out);
/* A2: level_out[v] (FP_NONE on/after a cycle), order_out = sort by (level, index).
 * n_cycle_out (nullable) receives the number of FP_NONE vertices. */
int fp_levelize(fp_ctx *ctx, const fp_graph *g, uint32_t *level_out, uint32_t *order_out,
                uint32_t *n_cycle_out);
/* A6: first-fit-decreasing; nodes mutated in place; level nullable. */
int fp_place(fp_ctx *ctx, const fp_containers *c, fp_nodes *nodes, const uint32_t *level,
             uint32_t *assign_out, uint8_t *reason_out);
int fp_place_batch(fp_ctx *ctx, const fp_batch *b);
/* Stage 2: first feasible node (FP_NONE) and feasible-node count per container on
 * the given node state; bitmap_out (nullable, ceil(C/64) * N words) holds
 * bit (c, n) at word [(c/64) * N + n], bit c % 64. */
int fp_feasibility(fp_ctx *ctx, const fp_containers *c, const fp_nodes *nodes,
                   uint32_t *first_out, uint32_t *count_out, uint64_t *bitmap_out);
/* One stage's whole plan, the `fleet up --dry-run` path (crates/fleetflow/src/commands/up.rs:57-136):
 *   perm_out                 A1 legacy start order (engine.rs:64-85, as fp_legacy_order)
 *   level_out, order_out, n_cycle_out   A2 levels and start order (as fp_levelize)
 * and, when nodes is not NULL (a stage with servers; c->n == n_vertices, container v = vertex v):
 *   first_out, count_out     stage 2 on the pristine table (as fp_feasibility; nullable)
 *   assign_out, reason_out   A6 first-fit-decreasing gated by the levels' CYCLE (as fp_place);
 *                            nodes updated in place.
 * A stage of <= 512 services, <= 8192 edges and <= 4096 servers is ONE kernel reading its inputs
 * from and writing its results to mapped pinned host memory (one launch and one synchronisation,
 * no copy calls: BASELINE config 1); larger stages run the general kernels.  FP_OPT_LEVEL_SMALL = 0
 * forces the general path.  Synchronous; on error nothing is written. */
int fp_plan_stage(fp_ctx *ctx, const fp_graph *g, const fp_containers *c, fp_nodes *nodes,
                  uint32_t *perm_out, uint32_t *level_out, uint32_t *order_out, uint32_t *n_cycle_out,
                  uint32_t *first_out, uint32_t *count_out, uint32_t *assign_out, uint8_t *reason_out);

/* ---- device-pointer API (async on the ctx stream) ----------------------- */
int fp_dev_legacy_order(fp_ctx *ctx, const fp_graph *g, uint32_t *perm_out);
int fp_dev_levelize(fp_ctx *ctx, const fp_graph *g, uint32_t *level_out, uint32_t *order_out,
                    uint32_t *n_cycle_out_dev);
int fp_dev_place_batch(fp_ctx *ctx, const fp_batch *b);
/* Device workspace (bytes) fp_place_batch / fp_dev_place_batch take on this ctx for
 * n_scen scenarios of n_containers x n_nodes (0 when there is nothing to place); the ctx
 * grows its workspace to it on the first such call and keeps it.  Depends on the device
 * (the pipeline's link sizing follows its occupancy). */
int fp_place_ws_bytes(fp_ctx *ctx, uint32_t n_scen, uint32_t n_containers, uint32_t n_nodes,
                      uint64_t *bytes_out);
/* The placement pipeline a batch of n_scen x n_containers x n_nodes runs on this ctx and
 * device (options included): out[FP_GEOM_*]. */
enum { FP_GEOM_GROUPS = 0, FP_GEOM_STAGES = 1, FP_GEOM_SEGMENTS = 2, FP_GEOM_RING = 3, FP_GEOM_LAG = 4,
       FP_GEOM_LINK_SLOTS = 5, FP_GEOM_BOUNDED = 6, FP_GEOM_RESIDENT = 7, FP_GEOM_SYSTOLIC = 8,
       FP_GEOM_COUNT = 9 };
int fp_place_geometry(fp_ctx *ctx, uint32_t n_scen, uint32_t n_containers, uint32_t n_nodes, uint32_t *out);
int fp_dev_feasibility(fp_ctx *ctx, const fp_containers *c, const fp_nodes *nodes,
                       uint32_t *first_out, uint32_t *count_out, uint64_t *bitmap_out);
/* Stage 2 batched over what-if scenarios: for each scenario s and container c of b
 * (b's containers and node state; nothing is placed or mutated), first_out[s*C + c] = the
 * lowest feasible node (FP_NONE if none) and count_out[s*C + c] = the number of feasible
 * nodes.  n_scen <= 65535. */
int fp_dev_feasibility_batch(fp_ctx *ctx, const fp_batch *b, uint32_t *first_out, uint32_t *count_out);
/* Best plan over a cost vector (device): writes the argmin index to *best_dev. */
int fp_dev_argmin_cost(fp_ctx *ctx, const uint64_t *cost, uint32_t n, uint32_t *best_dev);

/* ---- synthetic inputs (SPEC.md section 3), device-side ------------------- */
/* flags: bit0 host ports, bit1 anti-affinity groups, bit2 required labels. */
int fp_dev_gen_batch(fp_ctx *ctx, uint64_t seed, const fp_batch *b, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif
