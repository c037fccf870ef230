"""Control-plane server registry -> planner node table.

fleetflowd lists a tenant's servers with
``SELECT * FROM server WHERE tenant.slug = $t AND deleted_at IS NONE ORDER BY slug``
(crates/fleetflow-controlplane/src/db.rs:741-750). Each row carries optional
``capacity``/``allocated`` (model.rs:414-427), ``labels`` (model.rs:399-411) and
``scheduling`` (model.rs:435-442). The planner's node index is the position in
that slug order. The conversion is SPEC.md 4:

* ``cpu_free = (capacity.cpu_cores - allocated.cpu_cores) * 1000`` millicores;
* ``mem_free = (capacity.memory_gb - allocated.memory_gb) * 1024`` MiB;
* a missing capacity falls back to the plan string (``parse_plan``,
  crates/fleetflow-cloud-sakura/src/provider.rs:15-30), and a row with neither is
  unconstrained;
* ``scheduling`` other than "schedulable" (cordon, drain) makes the node
  unschedulable; None means schedulable (model.rs:516-518);
* labels become ``key=value`` strings (tier, region, class, arch, then the
  ``extras`` object), mapped to bits by ``flow.LabelDict``.
"""
from __future__ import annotations

from .flow import U32_MAX, Server

SCHEDULABLE, CORDON, DRAIN = "schedulable", "cordon", "drain"


def _rust_i32(s: str):
    """``str::parse::<i32>()``: optional sign, ASCII digits only, in range."""
    if not s:
        return None
    body = s[1:] if s[0] in "+-" else s
    if not body or not all("0" <= ch <= "9" for ch in body):
        return None
    v = int(s)
    return v if -(2 ** 31) <= v < 2 ** 31 else None


def _trim_end_matches(s: str, suffix: str) -> str:
    while suffix and s.endswith(suffix):
        s = s[:-len(suffix)]
    return s


def parse_plan(plan: str | None) -> tuple[int, int]:
    """provider.rs:15-30: ``"Ncore-Mgb"`` -> (N, M); any part that does not parse
    is 1, and anything but exactly two ``-`` parts is (1, 1)."""
    if plan is not None:
        parts = plan.split("-")
        if len(parts) == 2:
            core = _rust_i32(_trim_end_matches(parts[0], "core"))
            mem = _rust_i32(_trim_end_matches(parts[1], "gb"))
            return (1 if core is None else core, 1 if mem is None else mem)
    return (1, 1)


def _clamp_u32(v: int) -> int:
    return 0 if v < 0 else min(v, U32_MAX)


def server_labels(labels: dict | None) -> list[str]:
    if not labels:
        return []
    out = [f"{k}={labels[k]}" for k in ("tier", "region", "class", "arch") if labels.get(k) is not None]
    extras = labels.get("extras")
    if isinstance(extras, dict):
        out += [f"{k}={v}" for k, v in sorted(extras.items()) if isinstance(v, (str, int, float, bool))]
    return out


def server_from_row(row: dict) -> Server:
    """One registry ``server`` row (as JSON) -> planner node."""
    cap = row.get("capacity") or {}
    alloc = row.get("allocated") or {}
    cc, cm = cap.get("cpu_cores"), cap.get("memory_gb")
    if cc is None or cm is None:
        if row.get("plan") is not None:
            pc, pm = parse_plan(row["plan"])
            cc = pc if cc is None else cc
            cm = pm if cm is None else cm
    cpu = U32_MAX if cc is None else _clamp_u32((cc - (alloc.get("cpu_cores") or 0)) * 1000)
    mem = U32_MAX if cm is None else _clamp_u32((cm - (alloc.get("memory_gb") or 0)) * 1024)
    sched = row.get("scheduling")
    return Server(slug=row["slug"], cpu_m=cpu, mem_mib=mem, labels=server_labels(row.get("labels")),
                  schedulable=sched is None or sched == SCHEDULABLE, provider=row.get("provider", ""),
                  plan=row.get("plan"))


def node_table(rows: list[dict]) -> list[Server]:
    """db.rs:741-750: live rows (``deleted_at`` None) in slug order."""
    live = [r for r in rows if r.get("deleted_at") is None]
    return [server_from_row(r) for r in sorted(live, key=lambda r: r["slug"])]


def pool_required_labels(pool: dict | None) -> list[str]:
    """WorkerPool.required_labels (model.rs:557-558) -> required ``key=value`` labels."""
    req = (pool or {}).get("required_labels") or {}
    return [f"{k}={v}" for k, v in sorted(req.items())]
