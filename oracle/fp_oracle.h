/*
 * fp_oracle.h -- CPU ORACLE for the FleetFlow placement planner.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load or call this code, and only as the checker / the
 * timed CPU baseline.  The product (libfleetplace.so) never links or calls it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - fpo_legacy_order      : PINNED by the reference's own unit tests
 *                             crates/fleetflow-container/src/engine.rs:603-666
 *                             (restates engine.rs:67-85).
 *   - fpo_levelize          : new semantics (no reference implementation); pinned
 *                             against the reference only through the depth<=1
 *                             theorem (order == legacy order on the engine.rs tests).
 *   - fpo_place (FFD)       : new semantics, "parity unpinned" against the reference
 *                             beyond the N=1 special case that restates
 *                             crates/fleetflow-controlplane/src/handlers/deploy.rs:390-398.
 *   - generators            : SPEC.md section 3 (SplitMix64); pinned by the Python twin.
 *
 * Plain C11, single-threaded, deterministic.
 */
#ifndef FP_ORACLE_H
#define FP_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FPO_NONE 0xFFFFFFFFu
enum { FPO_OK = 0, FPO_NOFIT = 1, FPO_CYCLE = 2 };

/* A1: engine.rs:67-85 two-bucket stable partition.  has_deps[i] != 0 iff the
 * service is known in flow.services AND its depends_on is non-empty. */
void fpo_legacy_order(uint32_t n, const uint8_t *has_deps, uint32_t *perm_out);

/* A2: reference-compatible Kahn levels over a reversed CSR (dep -> dependent).
 * level(v) = max(has_deps(v), max_{d->v} level(d)+1); never-released vertices
 * (cycle members and everything downstream of a cycle) get FPO_NONE.
 * order_out = stable sort of 0..V-1 by (level, index), FPO_NONE last.
 * Returns the number of FPO_NONE vertices. */
uint32_t fpo_levelize(uint32_t V, const uint32_t *row_ptr, const uint32_t *col,
                      const uint8_t *has_deps, uint32_t *level_out, uint32_t *order_out);

/* FFD order: indices sorted by (cpu desc, mem desc, index asc). */
void fpo_ffd_order(uint32_t C, const uint32_t *cpu_m, const uint32_t *mem_mib, uint32_t *order_out);

/* A6: first-fit-decreasing.  Node arrays cpu_free/mem_free/conflict_used are
 * mutated in place.  level may be NULL.  assign_out[c] = node or FPO_NONE;
 * reason_out[c] = FPO_OK / FPO_NOFIT / FPO_CYCLE.  Returns #rejected.
 * If evals_out != NULL it receives the number of node records examined. */
uint32_t fpo_place(uint32_t C, const uint32_t *cpu_m, const uint32_t *mem_mib,
                   const uint32_t *req_labels, const uint32_t *conflict,
                   uint32_t N, uint32_t *cpu_free, uint32_t *mem_free,
                   const uint32_t *labels, uint32_t *conflict_used, const uint8_t *schedulable,
                   const uint32_t *level, uint32_t *assign_out, uint8_t *reason_out,
                   uint64_t *evals_out);

/* Static feasibility sweep (stage 2) on the given node state:
 * first_out[c] = lowest feasible node or FPO_NONE, count_out[c] = #feasible nodes,
 * bitmap (optional, may be NULL): bit (c, n) at word [(c/64) * N + n], bit c%64. */
void fpo_feasibility(uint32_t C, const uint32_t *cpu_m, const uint32_t *mem_mib,
                     const uint32_t *req_labels, const uint32_t *conflict,
                     uint32_t N, const uint32_t *cpu_free, const uint32_t *mem_free,
                     const uint32_t *labels, const uint32_t *conflict_used, const uint8_t *schedulable,
                     uint32_t *first_out, uint32_t *count_out, uint64_t *bitmap_out);

/* Packed plan cost: (n_rejected:24 | n_nodes_used:24 | scenario_id:16). */
uint64_t fpo_cost(uint32_t C, const uint32_t *assign, uint32_t N, uint32_t scenario_id);

/* ---- SPEC.md section 3 synthetic generators (SplitMix64, counter form) ---- */
uint64_t fpo_splitmix_draw(uint64_t seed, uint64_t idx);
uint64_t fpo_scenario_seed(uint64_t seed, uint32_t scenario);
/* flags: bit0 ports, bit1 anti-affinity, bit2 required labels */
void fpo_gen_containers(uint64_t seed, uint32_t C, uint32_t flags,
                        uint32_t *cpu_m, uint32_t *mem_mib, uint32_t *req_labels, uint32_t *conflict);
void fpo_gen_nodes(uint64_t seed, uint32_t N, uint32_t flags,
                   uint32_t *cpu_free, uint32_t *mem_free, uint32_t *labels,
                   uint32_t *conflict_used, uint8_t *schedulable);
/* Config-5 DAG.  Returns E; fills row_ptr[V+1], col[E] (reversed CSR), has_deps[V].
 * Call with col == NULL first to get E (row_ptr/has_deps still filled). */
uint32_t fpo_gen_dag(uint64_t seed, uint32_t n_chains, uint32_t chain_len,
                     uint32_t n_layers, uint32_t layer_width, uint32_t n_cycles,
                     uint32_t *row_ptr, uint32_t *col, uint8_t *has_deps);
uint32_t fpo_dag_vertices(uint32_t n_chains, uint32_t chain_len, uint32_t n_layers, uint32_t layer_width);

#ifdef __cplusplus
}
#endif
#endif
