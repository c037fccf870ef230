//! fleetflow-placement: FleetFlow's plan path on an MI355X (HIP/gfx950, libfleetplace.so).
//!
//! Drop-in replacements for the three seams of the reference:
//! * [`order_by_dependencies`] -- same signature and output as
//!   `fleetflow_container::order_by_dependencies` (crates/fleetflow-container/src/engine.rs:64-85),
//!   for the call at engine.rs:157;
//! * [`start_levels`] / [`start_waves`] -- Kahn start levels, the parallel start waves for
//!   `DeployEngine::create_and_start` (engine.rs:355-452);
//! * [`resolve_target_server`] / [`Planner::place`] -- the server choice of
//!   crates/fleetflow-controlplane/src/handlers/deploy.rs:390-398 (`servers.first()`), and the
//!   first-fit-decreasing fan-out that replaces it.
//!
//! Strings never cross the ABI: names map to u32 ids in stage order here.  There is no CPU
//! fallback: without an MI355X every call returns [`PlanError`] (FP_EDEVICE).
pub mod ffi;

use fleetflow_core::Flow;
use std::cell::RefCell;
use std::collections::HashMap;
use std::ffi::CStr;
use std::fmt;

/// A negative FP_E* code from libfleetplace.
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct PlanError(pub i32);

impl fmt::Display for PlanError {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        let msg = unsafe { CStr::from_ptr(ffi::fp_strerror(self.0)) };
        write!(f, "fleetplace: {} ({})", msg.to_string_lossy(), self.0)
    }
}
impl std::error::Error for PlanError {}

fn check(rc: i32) -> Result<(), PlanError> {
    if rc == ffi::FP_OK { Ok(()) } else { Err(PlanError(rc)) }
}

/// One planner context: a HIP stream on one MI355X.  Not shared between threads
/// (fleetplace.h: one fp_ctx per host thread); [`with_planner`] keeps one per thread.
pub struct Planner {
    ctx: *mut ffi::fp_ctx,
}

impl Planner {
    pub fn new(device: i32) -> Result<Self, PlanError> {
        let mut ctx = std::ptr::null_mut();
        check(unsafe { ffi::fp_ctx_create(&mut ctx, device) })?;
        Ok(Planner { ctx })
    }

    /// engine.rs:67-85 on indices: `has_deps[i]` = known in flow.services AND depends_on
    /// non-empty; returns the stable two-bucket permutation.
    pub fn legacy_order(&mut self, has_deps: &[u8]) -> Result<Vec<u32>, PlanError> {
        let g = ffi::fp_graph { n_vertices: has_deps.len() as u32, n_edges: 0, row_ptr: std::ptr::null(),
                                col: std::ptr::null(), has_deps: has_deps.as_ptr() };
        let mut perm = vec![0u32; has_deps.len()];
        check(unsafe { ffi::fp_legacy_order(self.ctx, &g, perm.as_mut_ptr()) })?;
        Ok(perm)
    }

    /// Kahn levels of a reversed CSR (SPEC.md 2.2): (level per vertex, FP_NONE on/after a
    /// cycle; order by (level, index); number of cycle vertices).
    pub fn levelize(&mut self, row_ptr: &[u32], col: &[u32], has_deps: &[u8])
                    -> Result<(Vec<u32>, Vec<u32>, u32), PlanError> {
        let v = has_deps.len();
        let g = ffi::fp_graph { n_vertices: v as u32, n_edges: col.len() as u32, row_ptr: row_ptr.as_ptr(),
                                col: if col.is_empty() { std::ptr::null() } else { col.as_ptr() },
                                has_deps: has_deps.as_ptr() };
        let (mut level, mut order, mut ncyc) = (vec![0u32; v], vec![0u32; v], 0u32);
        check(unsafe { ffi::fp_levelize(self.ctx, &g, level.as_mut_ptr(), order.as_mut_ptr(), &mut ncyc) })?;
        Ok((level, order, ncyc))
    }

    /// First-fit-decreasing placement (SPEC.md 2.3); `nodes` is updated in place.
    /// Returns (assign per container, FP_NONE if unplaced; reason per container).
    pub fn place(&mut self, c: &Containers, nodes: &mut Nodes, level: Option<&[u32]>)
                 -> Result<(Vec<u32>, Vec<u8>), PlanError> {
        let n = c.cpu_m.len();
        let cs = ffi::fp_containers { n: n as u32, cpu_m: c.cpu_m.as_ptr(), mem_mib: c.mem_mib.as_ptr(),
                                      req_labels: c.req_labels.as_ptr(), conflict: c.conflict.as_ptr() };
        let mut ns = ffi::fp_nodes { n: nodes.cpu_free.len() as u32, cpu_free: nodes.cpu_free.as_mut_ptr(),
                                     mem_free: nodes.mem_free.as_mut_ptr(), labels: nodes.labels.as_ptr(),
                                     conflict_used: nodes.conflict_used.as_mut_ptr(),
                                     schedulable: nodes.schedulable.as_ptr() };
        let (mut assign, mut reason) = (vec![0u32; n], vec![0u8; n]);
        check(unsafe {
            ffi::fp_place(self.ctx, &cs, &mut ns, level.map_or(std::ptr::null(), |l| l.as_ptr()),
                          assign.as_mut_ptr(), reason.as_mut_ptr())
        })?;
        Ok((assign, reason))
    }
}

impl Drop for Planner {
    fn drop(&mut self) {
        unsafe { ffi::fp_ctx_destroy(self.ctx) }
    }
}

/// Container requests (SoA): millicores, MiB, required label bits, conflict bits
/// (host-port bits 0-15 | anti-affinity group bits 16-31).
pub struct Containers {
    pub cpu_m: Vec<u32>,
    pub mem_mib: Vec<u32>,
    pub req_labels: Vec<u32>,
    pub conflict: Vec<u32>,
}

/// Node table (SoA) in node-index order (`stage.servers` order, or `ORDER BY slug` for
/// the controlplane registry, db.rs:741-750).
pub struct Nodes {
    pub cpu_free: Vec<u32>,
    pub mem_free: Vec<u32>,
    pub labels: Vec<u32>,
    pub conflict_used: Vec<u32>,
    pub schedulable: Vec<u8>,
}

thread_local! {
    static PLANNER: RefCell<Option<Planner>> = const { RefCell::new(None) };
}

/// Runs `f` with this thread's planner on device 0 (created on first use).
pub fn with_planner<R>(f: impl FnOnce(&mut Planner) -> Result<R, PlanError>) -> Result<R, PlanError> {
    PLANNER.with(|p| {
        let mut p = p.borrow_mut();
        if p.is_none() {
            *p = Some(Planner::new(0)?);
        }
        f(p.as_mut().unwrap())
    })
}

/// engine.rs:71-80 predicate per position: known in `flow.services` AND depends_on non-empty.
fn has_deps_vector(services: &[String], flow: &Flow) -> Vec<u8> {
    services.iter().map(|n| flow.services.get(n).map_or(0, |s| (!s.depends_on.is_empty()) as u8)).collect()
}

/// Same signature and output as `fleetflow_container::order_by_dependencies`
/// (crates/fleetflow-container/src/engine.rs:64-85), computed by the GPU planner.
/// Panics when no MI355X is available (the reference function is infallible; use
/// [`try_order_by_dependencies`] to handle the error).
pub fn order_by_dependencies(services: &[String], flow: &Flow) -> Vec<String> {
    try_order_by_dependencies(services, flow).expect("fleetflow-placement: GPU planner unavailable")
}

pub fn try_order_by_dependencies(services: &[String], flow: &Flow) -> Result<Vec<String>, PlanError> {
    if services.is_empty() {
        return Ok(Vec::new());
    }
    let perm = with_planner(|p| p.legacy_order(&has_deps_vector(services, flow)))?;
    Ok(perm.iter().map(|&i| services[i as usize].clone()).collect())
}

/// Reversed CSR of a stage's `depends_on` graph (SPEC.md 1): vertex = first occurrence of a
/// name in stage order; deps outside the stage add no edge; duplicate deps give duplicate
/// edges.  Returns (vertex of each position, row_ptr, col, has_deps per vertex).
pub fn stage_graph(services: &[String], flow: &Flow) -> (Vec<u32>, Vec<u32>, Vec<u32>, Vec<u8>) {
    let mut vid: HashMap<&str, u32> = HashMap::new();
    let mut names: Vec<&str> = Vec::new();
    let pos: Vec<u32> = services.iter().map(|n| *vid.entry(n.as_str()).or_insert_with(|| {
        names.push(n.as_str());
        (names.len() - 1) as u32
    })).collect();
    let v = names.len();
    let mut has_deps = vec![0u8; v];
    let mut edges: Vec<(u32, u32)> = Vec::new();
    for (i, n) in names.iter().enumerate() {
        if let Some(svc) = flow.services.get(*n) {
            if !svc.depends_on.is_empty() {
                has_deps[i] = 1;
                for d in &svc.depends_on {
                    if let Some(&dv) = vid.get(d.as_str()) {
                        edges.push((dv, i as u32));
                    }
                }
            }
        }
    }
    let mut row_ptr = vec![0u32; v + 1];
    for &(d, _) in &edges {
        row_ptr[d as usize + 1] += 1;
    }
    for i in 0..v {
        row_ptr[i + 1] += row_ptr[i];
    }
    let mut fill = row_ptr[..v].to_vec();
    let mut col = vec![0u32; edges.len()];
    for &(d, t) in &edges {
        col[fill[d as usize] as usize] = t;
        fill[d as usize] += 1;
    }
    (pos, row_ptr, col, has_deps)
}

/// Kahn start level of every position of `services` (`None` = CYCLE: the reference's
/// never-constructed `FlowError::CircularDependency`, crates/fleetflow-core/src/error.rs:42-43).
pub fn start_levels(services: &[String], flow: &Flow) -> Result<Vec<Option<u32>>, PlanError> {
    if services.is_empty() {
        return Ok(Vec::new());
    }
    let (pos, row_ptr, col, has_deps) = stage_graph(services, flow);
    let (level, _, _) = with_planner(|p| p.levelize(&row_ptr, &col, &has_deps))?;
    Ok(pos.iter().map(|&v| match level[v as usize] { ffi::FP_NONE => None, l => Some(l) }).collect())
}

/// Parallel start waves for `DeployEngine::create_and_start` (engine.rs:355-452): wave k holds
/// the services at level k, in declaration order; every in-stage dependency of a wave-k
/// service is in an earlier wave.  CYCLE services are in no wave (returned separately).
pub fn start_waves(services: &[String], flow: &Flow) -> Result<(Vec<Vec<String>>, Vec<String>), PlanError> {
    let levels = start_levels(services, flow)?;
    let mut by_level: std::collections::BTreeMap<u32, Vec<String>> = Default::default();
    let mut cycle = Vec::new();
    let mut seen = std::collections::HashSet::new();
    for (name, lv) in services.iter().zip(levels) {
        if !seen.insert(name.as_str()) {
            continue;
        }
        match lv {
            Some(l) => by_level.entry(l).or_default().push(name.clone()),
            None => cycle.push(name.clone()),
        }
    }
    Ok((by_level.into_values().collect(), cycle))
}

/// crates/fleetflow-controlplane/src/handlers/deploy.rs:390-394:
/// `flow.stages.get(stage).and_then(|s| s.servers.first().cloned())`, computed as FFD over the
/// stage's servers with unconstrained capacity (every service lands on node 0).  `None` means
/// the caller's "local" fallback (:396-398).
pub fn resolve_target_server(flow: &Flow, stage_name: &str) -> Result<Option<String>, PlanError> {
    let Some(stage) = flow.stages.get(stage_name) else { return Ok(None) };
    if stage.servers.is_empty() {
        return Ok(None);
    }
    let n = stage.services.len().max(1);
    let k = stage.servers.len();
    let c = Containers { cpu_m: vec![0; n], mem_mib: vec![0; n], req_labels: vec![0; n], conflict: vec![0; n] };
    let mut nodes = Nodes { cpu_free: vec![u32::MAX; k], mem_free: vec![u32::MAX; k], labels: vec![0; k],
                            conflict_used: vec![0; k], schedulable: vec![1; k] };
    let (assign, _) = with_planner(|p| p.place(&c, &mut nodes, None))?;
    Ok(Some(stage.servers[assign[0] as usize].clone()))
}

#[cfg(all(test, feature = "gpu-tests"))]
mod tests {
    //! The reference's own known answers (engine.rs:603-666), on the GPU.
    use super::*;
    use fleetflow_core::{Flow, Service};

    fn flow(deps: &[(&str, &[&str])]) -> Flow {
        let mut f = Flow { name: "t".into(), services: Default::default(), stages: Default::default(),
                           providers: Default::default(), servers: Default::default(), registry: None,
                           variables: Default::default(), tenant: None };
        for (n, d) in deps {
            let mut s = Service::default();
            s.depends_on = d.iter().map(|x| x.to_string()).collect();
            f.services.insert(n.to_string(), s);
        }
        f
    }
    fn names(v: &[&str]) -> Vec<String> { v.iter().map(|s| s.to_string()).collect() }

    #[test]
    fn order_no_deps() {
        let f = flow(&[("web", &[]), ("db", &[])]);
        assert_eq!(order_by_dependencies(&names(&["web", "db"]), &f), names(&["web", "db"]));
    }

    #[test]
    fn order_with_deps() {
        let f = flow(&[("web", &["db"]), ("db", &[])]);
        assert_eq!(order_by_dependencies(&names(&["web", "db"]), &f), names(&["db", "web"]));
    }

    #[test]
    fn order_mixed() {
        let f = flow(&[("api", &["db"]), ("db", &[]), ("redis", &[]), ("worker", &["redis", "db"])]);
        let out = order_by_dependencies(&names(&["api", "db", "redis", "worker"]), &f);
        assert_eq!(out, names(&["db", "redis", "api", "worker"]));
    }

    #[test]
    fn waves_cross_every_edge() {
        let f = flow(&[("c", &["b"]), ("b", &["a"]), ("a", &[])]);
        let (waves, cycle) = start_waves(&names(&["c", "b", "a"]), &f).unwrap();
        assert_eq!(waves, vec![names(&["a"]), names(&["b"]), names(&["c"])]);
        assert!(cycle.is_empty());
    }
}
