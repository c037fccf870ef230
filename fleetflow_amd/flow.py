"""Host-side mirror of the reference's plan-path interface.

Names and argument meaning follow the Rust reference so callers (and tests) read
the same:

* ``Service`` / ``Stage`` / ``Flow``: the subset of fleetflow-core's model the
  plan path reads (crates/fleetflow-core/src/model/service.rs:26-70,
  model/stage.rs:48-64, model/flow.rs:15-41), plus the resource-request
  extension of SPEC.md 4 (``cpu_m``/``mem_mib``/labels/ports/anti-affinity).
* ``order_by_dependencies(services, flow)``: engine.rs:64-85, computed by the
  GPU stable partition (fp_legacy_order).
* ``resolve_target_server(flow, stage_name)``: handlers/deploy.rs:390-394,
  computed by GPU FFD placement over the stage's servers with unconstrained
  capacity (every container lands on node 0 == ``servers.first()``).
* ``levelize_stage`` / ``plan_stage``: the new planner outputs (SPEC.md 2).

Strings never cross the C ABI: names are mapped to u32 ids in stage order here.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .planner import NONE, Planner

U32_MAX = 0xFFFFFFFF


@dataclass
class Port:
    """fleetflow_core::Port (model/port.rs); parsed by parser/port.rs."""
    host: int
    container: int
    protocol: str = "tcp"
    host_ip: str | None = None


@dataclass
class Volume:
    """fleetflow_core::Volume (model/volume.rs); parsed by parser/volume.rs."""
    host: str
    container: str
    read_only: bool = False


@dataclass
class Service:
    """fleetflow_core::Service subset (model/service.rs:26-70): the fields the plan
    path and the dry-run presenter read."""
    image: str | None = None
    version: str | None = None
    command: str | None = None
    service_type: str | None = None
    restart: str | None = None
    registry: str | None = None
    ports: list[Port] = field(default_factory=list)
    environment: dict[str, str] = field(default_factory=dict)
    volumes: list[Volume] = field(default_factory=list)
    depends_on: list[str] = field(default_factory=list)
    # SPEC.md 4 resource-request extension (ignored by the reference parser,
    # parser/service.rs:222); absent => unconstrained (0)
    cpu_m: int = 0
    mem_mib: int = 0
    labels: list[str] = field(default_factory=list)      # required "key=value" labels
    anti_affinity: str | None = None

    @property
    def host_ports(self) -> list[int]:
        return [p.host for p in self.ports]

    def merge(self, other: "Service") -> None:
        """model/service.rs:380-428: Options override when set, Vecs when non-empty,
        the environment map is merged with ``other`` winning."""
        for f in ("service_type", "image", "version", "command", "restart", "registry", "anti_affinity"):
            if getattr(other, f) is not None:
                setattr(self, f, getattr(other, f))
        for f in ("ports", "volumes", "depends_on", "labels"):
            if getattr(other, f):
                setattr(self, f, list(getattr(other, f)))
        for f in ("cpu_m", "mem_mib"):
            if getattr(other, f):
                setattr(self, f, getattr(other, f))
        self.environment.update(other.environment)


@dataclass
class Stage:
    """fleetflow_core::Stage (model/stage.rs:48-64)."""
    services: list[str] = field(default_factory=list)
    servers: list[str] = field(default_factory=list)
    variables: dict[str, str] = field(default_factory=dict)
    registry: str | None = None
    backend: str = "docker"


@dataclass
class Server:
    """Node-table entry: KDL ``server`` (parser/cloud.rs:46-140) or a CP registry
    row (controlplane model.rs:399-442 capacity/labels/scheduling)."""
    slug: str
    cpu_m: int = U32_MAX
    mem_mib: int = U32_MAX
    labels: list[str] = field(default_factory=list)
    schedulable: bool = True
    provider: str = ""
    plan: str | None = None


@dataclass
class Flow:
    """fleetflow_core::Flow subset (model/flow.rs:15-41)."""
    name: str = ""
    services: dict[str, Service] = field(default_factory=dict)
    stages: dict[str, Stage] = field(default_factory=dict)
    servers: dict[str, Server] = field(default_factory=dict)
    registry: str | None = None
    variables: dict[str, str] = field(default_factory=dict)


_PLANNER: Planner | None = None


def default_planner() -> Planner:
    global _PLANNER
    if _PLANNER is None:
        _PLANNER = Planner(0)
    return _PLANNER


def has_deps_vector(services: list[str], flow: Flow) -> np.ndarray:
    """The engine.rs:71-80 predicate per position: known AND depends_on non-empty."""
    return np.array([1 if (n in flow.services and flow.services[n].depends_on) else 0 for n in services],
                    dtype=np.uint8)


def order_by_dependencies(services: list[str], flow: Flow, planner: Planner | None = None) -> list[str]:
    """engine.rs:64-85 -- same inputs, same output, computed on the GPU."""
    if not services:
        return []
    p = planner or default_planner()
    perm = p.legacy_order(has_deps_vector(services, flow))
    return [services[i] for i in perm]


def stage_graph(services: list[str], flow: Flow):
    """Target set -> reversed CSR.

    Vertex ids: first occurrence of each name in stage order.  Deps outside the
    target set add no edge (they count as satisfied).  Duplicate deps give
    duplicate edges.  Returns (vertex_names, pos_to_vertex, row_ptr, col, has_deps)."""
    names, pos_to_vertex, row_ptr, col, has_deps = stage_graph_lists(services, flow)
    return (names, np.array(pos_to_vertex, np.uint32), np.array(row_ptr, np.uint32), np.array(col, np.uint32),
            np.frombuffer(has_deps, np.uint8))


def stage_graph_lists(services: list[str], flow: Flow):
    """stage_graph as plain lists (pos_to_vertex, row_ptr, col) and a bytearray (has_deps)."""
    vid: dict[str, int] = {}
    names: list[str] = []
    pos_to_vertex = []
    for n in services:
        if n not in vid:
            vid[n] = len(names)
            names.append(n)
        pos_to_vertex.append(vid[n])
    V = len(names)
    # plain lists, one array conversion each at the end: a fleet.kdl stage has a handful of services,
    # where per-element numpy indexing costs more than the graph (config 1 is timed per plan)
    has_deps = bytearray(V)
    edges = []
    for v, n in enumerate(names):
        svc = flow.services.get(n)
        if svc is None or not svc.depends_on:
            continue
        has_deps[v] = 1
        for d in svc.depends_on:
            u = vid.get(d)
            if u is not None:
                edges.append((u, v))
    row_ptr = [0] * (V + 1)
    for d, _ in edges:
        row_ptr[d + 1] += 1
    for i in range(V):
        row_ptr[i + 1] += row_ptr[i]
    col = [0] * len(edges)
    fill = row_ptr[:-1]
    for d, v in edges:
        col[fill[d]] = v
        fill[d] += 1
    return names, pos_to_vertex, row_ptr, col, has_deps


def levelize_stage(services: list[str], flow: Flow, planner: Planner | None = None):
    """Kahn start levels per position and the (level, position) start order."""
    if not services:
        return [], []
    p = planner or default_planner()
    names, pos2v, row_ptr, col, has_deps = stage_graph(services, flow)
    level_v, _, _ = p.levelize(row_ptr, col, has_deps)
    levels = [int(level_v[v]) for v in pos2v]
    order = sorted(range(len(services)), key=lambda i: (levels[i] == NONE, levels[i], i))
    return levels, [services[i] for i in order]


class LabelDict:
    """Sorted (key=value) dictionary -> bit index, <= 32 labels."""

    def __init__(self, labels):
        self.bits = {lab: i for i, lab in enumerate(sorted(set(labels)))}
        if len(self.bits) > 32:
            raise ValueError("more than 32 distinct labels")

    def mask(self, labels):
        m = 0
        for lab in labels:
            m |= 1 << self.bits[lab]
        return m


@dataclass
class Plan:
    stage: str
    order: list[str]              # legacy-compatible start order (engine.rs:67-85)
    levels: dict[str, int]        # Kahn levels (U32_MAX = cycle)
    level_order: list[str]        # sort by (level, position)
    assignment: dict[str, str]    # service -> server slug (unplaced absent)
    rejected: dict[str, str]      # service -> "NOFIT" | "CYCLE"
    # stage 2 on the stage's pristine server table: service -> (feasible servers, first feasible
    # slug or None); count 0 is an exact NOFIT before placement (SPEC.md 2.3 monotonicity)
    candidates: dict[str, tuple[int, str | None]] = field(default_factory=dict)


def _server_nodes(flow: Flow, servers: list[str]):
    out = []
    for s in servers:
        out.append(flow.servers.get(s, Server(slug=s)))
    return out


def _stage_tables(names: list[str], flow: Flow, nodes: list[Server]):
    """The stage's services (vertex order) and servers as the SoA tables of the C ABI: label,
    host-port and anti-affinity bit dictionaries (SPEC.md 4)."""
    svcs = [flow.services.get(n, Service()) for n in names]
    all_labels = [lab for s in svcs for lab in s.labels] + [lab for nd in nodes for lab in nd.labels]
    ld = LabelDict(all_labels)
    ports = sorted({hp for s in svcs for hp in s.host_ports})
    groups = sorted({s.anti_affinity for s in svcs if s.anti_affinity})
    if len(ports) > 16 or len(groups) > 16:
        raise ValueError("more than 16 host ports or anti-affinity groups in one stage")
    pbit = {hp: i for i, hp in enumerate(ports)}
    gbit = {g: 16 + i for i, g in enumerate(groups)}
    cpu = [s.cpu_m for s in svcs]
    mem = [s.mem_mib for s in svcs]
    req = [ld.mask(s.labels) for s in svcs]
    conf = []
    for s in svcs:
        m = 0
        for hp in s.host_ports:
            m |= 1 << pbit[hp]
        if s.anti_affinity:
            m |= 1 << gbit[s.anti_affinity]
        conf.append(m)
    cf = [nd.cpu_m for nd in nodes]
    mf = [nd.mem_mib for nd in nodes]
    lab = [ld.mask(nd.labels) for nd in nodes]
    cu = [0] * len(nodes)
    sch = [1 if nd.schedulable else 0 for nd in nodes]
    return (cpu, mem, req, conf), (cf, mf, lab, cu, sch)


def plan_stage(flow: Flow, stage_name: str, planner: Planner | None = None,
               servers: list[Server] | None = None) -> Plan:
    """Full planner output for one stage (SPEC.md 2): the `fleet up --dry-run`
    plan (up.rs:57-136).  One fp_plan_stage call -- A1 order, A2 levels, and with servers the stage-2
    candidates and the FFD plan -- when every service name appears once in the stage; a stage
    listing a name twice (positions != vertices) takes the per-output calls."""
    p = planner or default_planner()
    stage = flow.stages[stage_name]
    services = list(stage.services)
    nodes = servers if servers is not None else _server_nodes(flow, stage.servers)
    assignment, rejected, candidates = {}, {}, {}
    if not services:
        return Plan(stage_name, [], {}, [], assignment, rejected, candidates)
    if not nodes:
        # no servers (the fleet.kdl fixtures): the graph stays in lists, one prebuilt call
        names, pos2v, row_ptr, col, has_deps = stage_graph_lists(services, flow)
        if len(names) == len(services):
            perm, levels, order_v, _ = p.plan_stage_lists(row_ptr, col, has_deps)
            return Plan(stage_name, [services[i] for i in perm], dict(zip(services, levels)),
                        [services[i] for i in order_v], assignment, rejected, candidates)
    names, pos2v, row_ptr, col, has_deps = stage_graph(services, flow)
    if len(names) == len(services):
        cont, ntab = _stage_tables(names, flow, nodes) if nodes else (None, None)
        perm, level_v, order_v, _, placed = p.plan_stage(row_ptr, col, has_deps, cont, ntab)
        order = [services[i] for i in perm.tolist()]
        levels = level_v.tolist()
        level_order = [services[i] for i in order_v.tolist()]
    else:
        order = order_by_dependencies(services, flow, p)
        levels, level_order = levelize_stage(services, flow, p)
        placed = None
        if nodes:
            lvl_v = {names[v]: levels[i] for i, v in enumerate(pos2v)}
            cont, ntab = _stage_tables(names, flow, nodes)
            # stage 2 (fp_feasibility): feasible-server count and first feasible server per service
            first, count, _ = p.feasibility(cont, ntab, bitmap=False)
            assign, reason, _ = p.place(cont, ntab, level=[lvl_v[n] for n in names])
            placed = (first, count, assign, reason, None)
    if placed is not None:
        first, count, assign, reason, _ = placed
        candidates = {n: (int(count[v]), nodes[int(first[v])].slug if int(first[v]) != NONE else None)
                      for v, n in enumerate(names)}
        for v, n in enumerate(names):
            if assign[v] != NONE:
                assignment[n] = nodes[assign[v]].slug
            else:
                rejected[n] = "CYCLE" if reason[v] == 2 else "NOFIT"
    return Plan(stage_name, order, dict(zip(services, levels)), level_order, assignment, rejected, candidates)


def resolve_target_server(flow: Flow, stage_name: str, planner: Planner | None = None) -> str | None:
    """handlers/deploy.rs:390-394: ``flow.stages.get(stage).and_then(|s| s.servers.first().cloned())``.

    Computed as FFD over the stage's servers with unconstrained capacity: every
    service lands on node 0.  An empty or missing stage/server list gives None
    (the caller records "local", :396-398)."""
    stage = flow.stages.get(stage_name)
    if stage is None or not stage.servers:
        return None
    p = planner or default_planner()
    n = max(1, len(stage.services))
    nodes = ([U32_MAX] * len(stage.servers), [U32_MAX] * len(stage.servers), [0] * len(stage.servers),
             [0] * len(stage.servers), [1] * len(stage.servers))
    assign, _, _ = p.place(([0] * n, [0] * n, [0] * n, [0] * n), nodes)
    return stage.servers[int(assign[0])]
