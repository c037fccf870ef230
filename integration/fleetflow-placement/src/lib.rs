//! fleetflow-placement: FleetFlow's plan path on an MI355X (HIP/gfx950, libfleetplace.so).
//!
//! Drop-in replacements for the three seams of the reference:
//! * [`order_by_dependencies`] -- same signature and output as
//!   `fleetflow_container::order_by_dependencies` (crates/fleetflow-container/src/engine.rs:64-85),
//!   for the call at engine.rs:157;
//! * [`start_levels`] / [`start_waves`] -- Kahn start levels, the parallel start waves for
//!   `DeployEngine::create_and_start` (engine.rs:355-452);
//! * [`resolve_target_server`] -- the server choice of
//!   crates/fleetflow-controlplane/src/handlers/deploy.rs:390-398 (`servers.first()`), exactly
//!   as the reference computes it (no planning involved, no GPU needed), and
//!   [`Planner::place`] / [`place_stage`] -- the first-fit-decreasing fan-out that replaces it
//!   when server capacity matters;
//! * [`plan_scenarios`] / [`Planner::place_batch`] -- what-if planning: many independent
//!   scenarios in one call, a packed cost per scenario and the best plan, the single-host
//!   counterpart of the controlplane routing a deploy to one target (deploy.rs:441-451).
//!
//! Strings never cross the ABI: names map to u32 ids in stage order here.  There is no CPU
//! fallback for the planning calls: without an MI355X they return [`PlanError`] (FP_EDEVICE),
//! and [`order_by_dependencies`] panics like any use of the crate on a host without the GPU
//! it is built for.
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
        if v > 0 && row_ptr.len() != v + 1 {
            return Err(PlanError(ffi::FP_EINVAL));
        }
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
        // fp_place reads every container array for n elements and reads / writes every node
        // array for nodes.len(): a shorter Vec would be read out of bounds from safe code
        if !c.all_len(n) || !nodes.all_len(nodes.cpu_free.len()) || level.map_or(false, |l| l.len() != n) {
            return Err(PlanError(ffi::FP_EINVAL));
        }
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

    /// One stage's whole dry-run plan in one call (fleetplace.h `fp_plan_stage`, the
    /// `fleet up --dry-run` path of up.rs:57-136): the legacy order, the Kahn levels and start
    /// order and, with `placement = Some((containers, nodes))` (container v = vertex v), the
    /// stage-2 first feasible server and count per service and the FFD plan, `nodes` updated
    /// in place.  A stage of <= 512 services is one kernel launch.
    pub fn plan_stage(&mut self, row_ptr: &[u32], col: &[u32], has_deps: &[u8],
                      placement: Option<(&Containers, &mut Nodes)>) -> Result<StagePlan, PlanError> {
        let v = has_deps.len();
        if v > 0 && row_ptr.len() != v + 1 {
            return Err(PlanError(ffi::FP_EINVAL));
        }
        let g = ffi::fp_graph { n_vertices: v as u32, n_edges: col.len() as u32, row_ptr: row_ptr.as_ptr(),
                                col: if col.is_empty() { std::ptr::null() } else { col.as_ptr() },
                                has_deps: has_deps.as_ptr() };
        let mut out = StagePlan { perm: vec![0; v], level: vec![0; v], order: vec![0; v], n_cycle: 0,
                                  first: vec![], count: vec![], assign: vec![], reason: vec![] };
        let rc = match placement {
            None => unsafe {
                ffi::fp_plan_stage(self.ctx, &g, std::ptr::null(), std::ptr::null_mut(), out.perm.as_mut_ptr(),
                                   out.level.as_mut_ptr(), out.order.as_mut_ptr(), &mut out.n_cycle,
                                   std::ptr::null_mut(), std::ptr::null_mut(), std::ptr::null_mut(),
                                   std::ptr::null_mut())
            },
            Some((c, nodes)) => {
                if !c.all_len(v) || !nodes.all_len(nodes.cpu_free.len()) {
                    return Err(PlanError(ffi::FP_EINVAL));
                }
                let cs = ffi::fp_containers { n: v as u32, cpu_m: c.cpu_m.as_ptr(), mem_mib: c.mem_mib.as_ptr(),
                                              req_labels: c.req_labels.as_ptr(), conflict: c.conflict.as_ptr() };
                let mut ns = ffi::fp_nodes { n: nodes.cpu_free.len() as u32, cpu_free: nodes.cpu_free.as_mut_ptr(),
                                             mem_free: nodes.mem_free.as_mut_ptr(), labels: nodes.labels.as_ptr(),
                                             conflict_used: nodes.conflict_used.as_mut_ptr(),
                                             schedulable: nodes.schedulable.as_ptr() };
                out.first = vec![0; v];
                out.count = vec![0; v];
                out.assign = vec![0; v];
                out.reason = vec![0; v];
                unsafe {
                    ffi::fp_plan_stage(self.ctx, &g, &cs, &mut ns, out.perm.as_mut_ptr(), out.level.as_mut_ptr(),
                                       out.order.as_mut_ptr(), &mut out.n_cycle, out.first.as_mut_ptr(),
                                       out.count.as_mut_ptr(), out.assign.as_mut_ptr(), out.reason.as_mut_ptr())
                }
            }
        };
        check(rc)?;
        Ok(out)
    }
}

/// The result of [`Planner::plan_stage`], per vertex of the stage graph.  The placement
/// vectors are empty for a stage planned without servers.
pub struct StagePlan {
    /// A1 legacy start order (engine.rs:64-85)
    pub perm: Vec<u32>,
    /// A2 start level (FP_NONE = CYCLE) and the (level, index) start order
    pub level: Vec<u32>,
    pub order: Vec<u32>,
    pub n_cycle: u32,
    /// stage 2 on the pristine server table: first feasible server (FP_NONE) and count
    pub first: Vec<u32>,
    pub count: Vec<u32>,
    /// A6 FFD: server per service (FP_NONE if unplaced) and reason (FP_REASON_*)
    pub assign: Vec<u32>,
    pub reason: Vec<u8>,
}

impl Planner {
    /// What-if planning over `b.n_scen` independent scenarios (fleetplace.h `fp_place_batch`):
    /// every scenario's plan, its packed cost `(n_rejected:24 | n_nodes_used:24 | id:16)` and
    /// the updated node tables, in `b` (scenario-major arrays).
    pub fn place_batch(&mut self, b: &mut Batch) -> Result<(), PlanError> {
        let (s, c, n) = (b.n_scen as usize, b.n_containers as usize, b.n_nodes as usize);
        // every array fp_place_batch reads or writes must hold S * C (containers) or S * N (nodes)
        let ok = b.containers.all_len(s * c) && b.nodes.all_len(s * n)
            && b.level.as_ref().map_or(true, |l| l.len() == s * c);
        if !ok {
            return Err(PlanError(ffi::FP_EINVAL));
        }
        b.assign.resize(s * c, 0);
        b.reason.resize(s * c, 0);
        b.cost.resize(s, 0);
        let fb = ffi::fp_batch {
            n_scen: b.n_scen, scen_base: b.scen_base, n_containers: b.n_containers, n_nodes: b.n_nodes,
            cpu_m: b.containers.cpu_m.as_ptr(), mem_mib: b.containers.mem_mib.as_ptr(),
            req_labels: b.containers.req_labels.as_ptr(), conflict: b.containers.conflict.as_ptr(),
            level: b.level.as_ref().map_or(std::ptr::null(), |l| l.as_ptr()),
            cpu_free: b.nodes.cpu_free.as_mut_ptr(), mem_free: b.nodes.mem_free.as_mut_ptr(),
            labels: b.nodes.labels.as_ptr(), conflict_used: b.nodes.conflict_used.as_mut_ptr(),
            schedulable: b.nodes.schedulable.as_ptr(), assign: b.assign.as_mut_ptr(), reason: b.reason.as_mut_ptr(),
            cost: b.cost.as_mut_ptr(),
        };
        check(unsafe { ffi::fp_place_batch(self.ctx, &fb) })
    }

    /// The same planning on HBM-resident arrays (fleetplace.h `fp_dev_place_batch`, asynchronous
    /// on the context's stream), then the best scenario on the device
    /// (`fp_dev_argmin_cost` into `best_dev`).  Kernel errors surface at [`Planner::sync`].
    ///
    /// # Safety
    /// Every pointer in `b` and `best_dev` must be device memory of this context's GPU, sized as
    /// fleetplace.h documents, and stay valid until the stream has drained.
    pub unsafe fn dev_place_batch(&mut self, b: &ffi::fp_batch, best_dev: *mut u32) -> Result<(), PlanError> {
        check(ffi::fp_dev_place_batch(self.ctx, b))?;
        if !b.cost.is_null() && !best_dev.is_null() && b.n_scen > 0 {
            check(ffi::fp_dev_argmin_cost(self.ctx, b.cost, b.n_scen, best_dev))?;
        }
        Ok(())
    }

    /// Waits for the context's asynchronous calls and reports their first kernel error.
    pub fn sync(&mut self) -> Result<(), PlanError> {
        check(unsafe { ffi::fp_ctx_sync(self.ctx) })
    }

    /// Device workspace a batch of this shape takes (grown once per context, then reused).
    pub fn workspace_bytes(&mut self, n_scen: u32, n_containers: u32, n_nodes: u32) -> Result<u64, PlanError> {
        let mut bytes = 0u64;
        check(unsafe { ffi::fp_place_ws_bytes(self.ctx, n_scen, n_containers, n_nodes, &mut bytes) })?;
        Ok(bytes)
    }

    /// The placement pipeline a batch of this shape runs (`FP_GEOM_*` indices).
    pub fn geometry(&mut self, n_scen: u32, n_containers: u32, n_nodes: u32)
                    -> Result<[u32; ffi::FP_GEOM_COUNT], PlanError> {
        let mut out = [0u32; ffi::FP_GEOM_COUNT];
        check(unsafe { ffi::fp_place_geometry(self.ctx, n_scen, n_containers, n_nodes, out.as_mut_ptr()) })?;
        Ok(out)
    }

    /// A per-context option (`FP_OPT_*`; `FP_OPT_AUTO` restores the default).
    pub fn set_option(&mut self, option: i32, value: i64) -> Result<(), PlanError> {
        check(unsafe { ffi::fp_ctx_set_option(self.ctx, option, value) })
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

impl Containers {
    /// every array holds exactly `n` elements
    fn all_len(&self, n: usize) -> bool {
        self.cpu_m.len() == n && self.mem_mib.len() == n && self.req_labels.len() == n && self.conflict.len() == n
    }
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

impl Nodes {
    /// every array holds exactly `n` elements
    fn all_len(&self, n: usize) -> bool {
        self.cpu_free.len() == n && self.mem_free.len() == n && self.labels.len() == n
            && self.conflict_used.len() == n && self.schedulable.len() == n
    }
}

/// `n_scen` independent what-if scenarios of `n_containers` x `n_nodes`, scenario-major
/// (`containers.*[s * C + i]`, `nodes.*[s * N + j]`); outputs filled by [`Planner::place_batch`].
pub struct Batch {
    pub n_scen: u32,
    /// global id of scenario 0 in the packed costs (scen_base + n_scen <= 65536)
    pub scen_base: u32,
    pub n_containers: u32,
    pub n_nodes: u32,
    pub containers: Containers,
    pub nodes: Nodes,
    /// start levels ([S * C]); `FP_NONE` marks a CYCLE member, which is not placed
    pub level: Option<Vec<u32>>,
    pub assign: Vec<u32>,
    pub reason: Vec<u8>,
    pub cost: Vec<u64>,
}

/// The outcome of [`plan_scenarios`]: every scenario's packed cost, the best scenario (lowest
/// cost; the id field breaks ties towards the lowest id) and its plan.
pub struct ScenarioPlans {
    pub cost: Vec<u64>,
    pub best: u32,
    pub assign: Vec<u32>,
    pub reason: Vec<u8>,
}

/// Unpacks a packed scenario cost: (rejected containers, nodes used, scenario id).
pub fn unpack_cost(c: u64) -> (u32, u32, u32) {
    ((c >> 40) as u32, ((c >> 16) & 0xFF_FFFF) as u32, (c & 0xFFFF) as u32)
}

/// Plans every scenario of `b` on this thread's GPU and picks the best one (the what-if
/// surface of the controlplane: one target per deploy, deploy.rs:441-451).
pub fn plan_scenarios(b: &mut Batch) -> Result<ScenarioPlans, PlanError> {
    with_planner(|p| p.place_batch(b))?;
    let c = b.n_containers as usize;
    let best = b.cost.iter().enumerate().min_by_key(|&(i, &v)| (v, i)).map_or(0, |(i, _)| i);
    Ok(ScenarioPlans { cost: b.cost.clone(), best: best as u32, assign: b.assign[best * c..(best + 1) * c].to_vec(),
                       reason: b.reason[best * c..(best + 1) * c].to_vec() })
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

/// crates/fleetflow-controlplane/src/handlers/deploy.rs:390-394, as the reference computes it:
/// `flow.stages.get(stage).and_then(|s| s.servers.first().cloned())`.  `None` means the caller's
/// "local" fallback (:396-398).  Pure Rust: choosing the first declared server needs no planner
/// (and so no GPU); [`place_stage`] is the capacity-aware fan-out that replaces it.
pub fn resolve_target_server(flow: &Flow, stage_name: &str) -> Option<String> {
    flow.stages.get(stage_name).and_then(|s| s.servers.first().cloned())
}

/// Per-service server choice for a stage (the fan-out deploy.rs:388-389 leaves for later):
/// first-fit-decreasing of the stage's services (requests in `c`, stage order) over its servers
/// (`nodes`, `stage.servers` order), on the GPU.  Returns the server of every service, `None`
/// for one that fits nowhere (NOFIT).  With unconstrained capacity every service lands on the
/// first server, i.e. [`resolve_target_server`].
pub fn place_stage(flow: &Flow, stage_name: &str, c: &Containers, nodes: &mut Nodes)
                   -> Result<Vec<Option<String>>, PlanError> {
    let Some(stage) = flow.stages.get(stage_name) else { return Err(PlanError(ffi::FP_EINVAL)) };
    if nodes.cpu_free.len() != stage.servers.len() || c.cpu_m.len() != stage.services.len() {
        return Err(PlanError(ffi::FP_EINVAL));
    }
    let (assign, _) = with_planner(|p| p.place(c, nodes, None))?;
    Ok(assign.iter().map(|&a| if a == ffi::FP_NONE { None } else { Some(stage.servers[a as usize].clone()) }).collect())
}

/// What `fleet up --dry-run` prints for a stage (up.rs:57-136), planned in one call: the
/// reference's start order, the start level of every service (`None` = CYCLE) and, when the
/// stage has servers and `placement` carries their tables, each service's server.  A stage
/// whose service list repeats a name is planned per vertex (first occurrence) and mapped back.
pub fn dry_run_stage(services: &[String], flow: &Flow, placement: Option<(&Containers, &mut Nodes)>)
                     -> Result<(Vec<String>, Vec<Option<u32>>, Option<Vec<Option<u32>>>), PlanError> {
    if services.is_empty() {
        return Ok((Vec::new(), Vec::new(), placement.map(|_| Vec::new())));
    }
    let (pos, row_ptr, col, has_deps) = stage_graph(services, flow);
    let placed = placement.is_some();
    let plan = with_planner(|p| p.plan_stage(&row_ptr, &col, &has_deps, placement))?;
    // the legacy order runs over positions (engine.rs:64-85 keeps duplicates); without
    // duplicates positions and vertices coincide
    let order = if pos.len() == has_deps.len() {
        plan.perm.iter().map(|&i| services[i as usize].clone()).collect()
    } else {
        try_order_by_dependencies(services, flow)?
    };
    let levels = pos.iter().map(|&v| match plan.level[v as usize] { ffi::FP_NONE => None, l => Some(l) }).collect();
    let servers = placed.then(|| pos.iter().map(|&v| match plan.assign[v as usize] {
        ffi::FP_NONE => None,
        a => Some(a),
    }).collect());
    Ok((order, levels, servers))
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
    fn scenarios_pick_the_cheapest_plan() {
        // two scenarios of two containers on one node: scenario 1's node is too small for
        // one of them, so scenario 0 (nothing rejected) is the best plan
        let c = Containers { cpu_m: vec![500, 500, 500, 500], mem_mib: vec![64; 4], req_labels: vec![0; 4],
                             conflict: vec![0; 4] };
        let nodes = Nodes { cpu_free: vec![1000, 600], mem_free: vec![1024, 1024], labels: vec![0; 2],
                            conflict_used: vec![0; 2], schedulable: vec![1; 2] };
        let mut b = Batch { n_scen: 2, scen_base: 0, n_containers: 2, n_nodes: 1, containers: c, nodes, level: None,
                            assign: vec![], reason: vec![], cost: vec![] };
        let p = plan_scenarios(&mut b).unwrap();
        assert_eq!(p.best, 0);
        assert_eq!(unpack_cost(p.cost[1]), (1, 1, 1));
        assert_eq!(p.assign, vec![0, 0]);
    }

    #[test]
    fn waves_cross_every_edge() {
        let f = flow(&[("c", &["b"]), ("b", &["a"]), ("a", &[])]);
        let (waves, cycle) = start_waves(&names(&["c", "b", "a"]), &f).unwrap();
        assert_eq!(waves, vec![names(&["a"]), names(&["b"]), names(&["c"])]);
        assert!(cycle.is_empty());
    }
}
