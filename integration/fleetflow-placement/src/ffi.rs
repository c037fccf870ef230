//! Raw bindings of include/fleetplace.h (ABI version 1).  Every `#[repr(C)]` struct here
//! mirrors the C struct field for field; tests/test_rust_binding.py checks that they
//! stay in step with the header.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

pub const FP_ABI_VERSION: c_int = 1;
pub const FP_OK: c_int = 0;
pub const FP_EINVAL: c_int = -1;
pub const FP_ENOMEM: c_int = -2;
pub const FP_EDEVICE: c_int = -3;
pub const FP_EOVERFLOW: c_int = -4;
pub const FP_ECORRUPT: c_int = -5;
pub const FP_NONE: u32 = 0xFFFF_FFFF;
pub const FP_REASON_OK: u8 = 0;
pub const FP_REASON_NOFIT: u8 = 1;
pub const FP_REASON_CYCLE: u8 = 2;
pub const FP_K_PLACE: c_int = 0;
pub const FP_K_SORT: c_int = 1;
pub const FP_K_FEAS: c_int = 2;
pub const FP_K_LEVEL: c_int = 3;
pub const FP_K_GEN: c_int = 4;
pub const FP_OPT_AUTO: i64 = -1;
pub const FP_OPT_PIPE_W: c_int = 0;
pub const FP_OPT_PIPE_SEG: c_int = 1;
pub const FP_OPT_PIPE_R: c_int = 2;
pub const FP_OPT_PIPE_LAG: c_int = 3;
pub const FP_OPT_LINK_SLOTS: c_int = 4;
pub const FP_OPT_LINK_BOUNDED: c_int = 5;
pub const FP_OPT_PIPE_FLUSH: c_int = 6;
pub const FP_OPT_SPIN_TICKS: c_int = 7;
pub const FP_OPT_KPACK: c_int = 8;
pub const FP_OPT_SCEN_SORT: c_int = 9;
/// Ignored (kept for ABI stability): the radix path is segmented for S > 1, device-wide for S == 1.
pub const FP_OPT_SEGSORT: c_int = 10;
pub const FP_OPT_SYSTOLIC: c_int = 11;
pub const FP_OPT_LEVELIZE_SYNC: c_int = 12;
pub const FP_OPT_SYSTOLIC_EXTRA: c_int = 13;
pub const FP_OPT_SCREEN: c_int = 14;
pub const FP_OPT_PAYLOAD_LDS: c_int = 15;
pub const FP_OPT_SYSTOLIC_VALU: c_int = 16;
pub const FP_OPT_LINK_PUBLISH: c_int = 17;
pub const FP_OPT_LEVEL_SORT: c_int = 18;
pub const FP_OPT_LEVEL_SMALL: c_int = 19;
pub const FP_OPT_PIPE_PRIO: c_int = 20;
pub const FP_OPT_INDEG_BIN: c_int = 21;
pub const FP_OPT_PACKED: c_int = 22;
pub const FP_GEOM_GROUPS: usize = 0;
pub const FP_GEOM_STAGES: usize = 1;
pub const FP_GEOM_SEGMENTS: usize = 2;
pub const FP_GEOM_RING: usize = 3;
pub const FP_GEOM_LAG: usize = 4;
pub const FP_GEOM_LINK_SLOTS: usize = 5;
pub const FP_GEOM_BOUNDED: usize = 6;
pub const FP_GEOM_RESIDENT: usize = 7;
pub const FP_GEOM_SYSTOLIC: usize = 8;
pub const FP_GEOM_COUNT: usize = 9;

/// Opaque `fp_ctx` (one per host thread; owns a HIP stream on one MI355X).
#[repr(C)]
pub struct fp_ctx {
    _private: [u8; 0],
}

/// depends_on graph as a reversed CSR (row d lists the vertices depending on d).
#[repr(C)]
pub struct fp_graph {
    pub n_vertices: u32,
    pub n_edges: u32,
    pub row_ptr: *const u32,
    pub col: *const u32,
    pub has_deps: *const u8,
}

/// Container requests, SoA.
#[repr(C)]
pub struct fp_containers {
    pub n: u32,
    pub cpu_m: *const u32,
    pub mem_mib: *const u32,
    pub req_labels: *const u32,
    pub conflict: *const u32,
}

/// Node table, SoA, in node-index order; cpu_free/mem_free/conflict_used updated in place.
#[repr(C)]
pub struct fp_nodes {
    pub n: u32,
    pub cpu_free: *mut u32,
    pub mem_free: *mut u32,
    pub labels: *const u32,
    pub conflict_used: *mut u32,
    pub schedulable: *const u8,
}

/// S what-if scenarios, scenario-major arrays ([S][C] containers, [S][N] nodes).
#[repr(C)]
pub struct fp_batch {
    pub n_scen: u32,
    pub scen_base: u32,
    pub n_containers: u32,
    pub n_nodes: u32,
    pub cpu_m: *const u32,
    pub mem_mib: *const u32,
    pub req_labels: *const u32,
    pub conflict: *const u32,
    pub level: *const u32,
    pub cpu_free: *mut u32,
    pub mem_free: *mut u32,
    pub labels: *const u32,
    pub conflict_used: *mut u32,
    pub schedulable: *const u8,
    pub assign: *mut u32,
    pub reason: *mut u8,
    pub cost: *mut u64,
}

#[link(name = "fleetplace")]
unsafe extern "C" {
    pub fn fp_ctx_create(out: *mut *mut fp_ctx, device: c_int) -> c_int;
    pub fn fp_ctx_destroy(ctx: *mut fp_ctx);
    pub fn fp_ctx_set_stream(ctx: *mut fp_ctx, hip_stream: *mut c_void) -> c_int;
    pub fn fp_ctx_reset_stream(ctx: *mut fp_ctx) -> c_int;
    pub fn fp_ctx_sync(ctx: *mut fp_ctx) -> c_int;
    pub fn fp_strerror(code: c_int) -> *const c_char;
    pub fn fp_abi_version() -> c_int;
    pub fn fp_ctx_profile(ctx: *mut fp_ctx, enable: c_int) -> c_int;
    pub fn fp_ctx_kernel_stats(ctx: *mut fp_ctx, kernel_id: c_int, total_ms: *mut f64, launches: *mut u64) -> c_int;
    pub fn fp_ctx_place_path(ctx: *mut fp_ctx, out3: *mut u32) -> c_int;
    pub fn fp_ctx_set_option(ctx: *mut fp_ctx, option: c_int, value: i64) -> c_int;
    pub fn fp_ctx_get_option(ctx: *mut fp_ctx, option: c_int, value: *mut i64) -> c_int;

    pub fn fp_legacy_order(ctx: *mut fp_ctx, g: *const fp_graph, perm_out: *mut u32) -> c_int;
    pub fn fp_levelize(ctx: *mut fp_ctx, g: *const fp_graph, level_out: *mut u32, order_out: *mut u32,
                       n_cycle_out: *mut u32) -> c_int;
    pub fn fp_place(ctx: *mut fp_ctx, c: *const fp_containers, nodes: *mut fp_nodes, level: *const u32,
                    assign_out: *mut u32, reason_out: *mut u8) -> c_int;
    pub fn fp_place_batch(ctx: *mut fp_ctx, b: *const fp_batch) -> c_int;
    pub fn fp_feasibility(ctx: *mut fp_ctx, c: *const fp_containers, nodes: *const fp_nodes, first_out: *mut u32,
                          count_out: *mut u32, bitmap_out: *mut u64) -> c_int;
    pub fn fp_plan_stage(ctx: *mut fp_ctx, g: *const fp_graph, c: *const fp_containers, nodes: *mut fp_nodes,
                         perm_out: *mut u32, level_out: *mut u32, order_out: *mut u32, n_cycle_out: *mut u32,
                         first_out: *mut u32, count_out: *mut u32, assign_out: *mut u32, reason_out: *mut u8)
                         -> c_int;

    pub fn fp_dev_legacy_order(ctx: *mut fp_ctx, g: *const fp_graph, perm_out: *mut u32) -> c_int;
    pub fn fp_dev_levelize(ctx: *mut fp_ctx, g: *const fp_graph, level_out: *mut u32, order_out: *mut u32,
                           n_cycle_out_dev: *mut u32) -> c_int;
    pub fn fp_dev_place_batch(ctx: *mut fp_ctx, b: *const fp_batch) -> c_int;
    pub fn fp_place_ws_bytes(ctx: *mut fp_ctx, n_scen: u32, n_containers: u32, n_nodes: u32,
                             bytes_out: *mut u64) -> c_int;
    pub fn fp_place_geometry(ctx: *mut fp_ctx, n_scen: u32, n_containers: u32, n_nodes: u32,
                             out: *mut u32) -> c_int;
    pub fn fp_dev_feasibility(ctx: *mut fp_ctx, c: *const fp_containers, nodes: *const fp_nodes,
                              first_out: *mut u32, count_out: *mut u32, bitmap_out: *mut u64) -> c_int;
    pub fn fp_dev_feasibility_batch(ctx: *mut fp_ctx, b: *const fp_batch, first_out: *mut u32,
                                    count_out: *mut u32) -> c_int;
    pub fn fp_dev_argmin_cost(ctx: *mut fp_ctx, cost: *const u64, n: u32, best_dev: *mut u32) -> c_int;
    pub fn fp_dev_gen_batch(ctx: *mut fp_ctx, seed: u64, b: *const fp_batch, flags: u32) -> c_int;
}
