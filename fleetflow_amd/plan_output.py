"""Plan output: JSON plan and the dry-run presenter.

``plan_to_json`` is the machine form carried to the control plane next to
``DeployRequest`` (crates/fleetflow-container/src/engine.rs:16-25):
``{stage, order, levels, level_order, assign, rejected}``.

``format_up_dry_run`` / ``format_deploy_dry_run`` reproduce the reference's
``fleet up --dry-run`` (crates/fleetflow/src/commands/up.rs:57-136) and
``fleet deploy --dry-run`` (crates/fleetflow/src/commands/deploy.rs:14-100)
line for line, without ANSI colour. When a ``Plan`` is given, each service
block gains its start level, its candidate servers (stage 2: the feasible-server count
and the first feasible server on the pristine table) and its planned server. Without one the
text is the reference's. The environment line lists variables in definition
order (the reference iterates a HashMap, so its order is arbitrary; compare it
as a set).
"""
from __future__ import annotations

import json

from .flow import U32_MAX, Flow, Plan
from .parser import FlowError


def plan_to_json(plan: Plan, indent: int | None = None) -> str:
    """Serialise a plan; a cycle member's level is null (it was U32_MAX)."""
    return json.dumps({
        "stage": plan.stage,
        "order": plan.order,
        "levels": {k: (None if v == U32_MAX else v) for k, v in plan.levels.items()},
        "level_order": plan.level_order,
        "assign": plan.assignment,
        "rejected": plan.rejected,
        "candidates": {k: {"count": c, "first": f} for k, (c, f) in plan.candidates.items()},
    }, ensure_ascii=False, indent=indent)


def plan_from_json(text: str) -> Plan:
    d = json.loads(text)
    return Plan(d["stage"], d["order"], {k: (U32_MAX if v is None else v) for k, v in d["levels"].items()},
                d["level_order"], d["assign"], d["rejected"],
                {k: (v["count"], v["first"]) for k, v in d.get("candidates", {}).items()})


def get_network_name(project: str, stage: str) -> str:
    """crates/fleetflow-container/src/converter.rs:12-14."""
    return f"{project}-{stage}"


def is_sensitive_key(key: str) -> bool:
    """crates/fleetflow/src/utils.rs:76-82."""
    k = key.lower()
    return "pass" in k or "secret" in k or "key" in k or "token" in k


def _service_block(flow: Flow, stage: str, name: str, container_suffix: str, plan: Plan | None) -> list[str]:
    svc = flow.services.get(name)
    if svc is None:
        raise FlowError(f"サービス '{name}' の定義が見つかりません")
    lines = ["", f"  サービス: {name}",
             f"    コンテナ: {flow.name}-{stage}-{name}{container_suffix}",
             f"    イメージ: {svc.image if svc.image is not None else '(未設定)'}"]
    for p in svc.ports:
        lines.append(f"    ポート: {p.host} → {p.container}/{p.protocol}")
    for v in svc.volumes:
        lines.append(f"    ボリューム: {v.host} → {v.container} ({'ro' if v.read_only else 'rw'})")
    if svc.environment:
        env = [f"{k}=***" if is_sensitive_key(k) else f"{k}={v}" for k, v in svc.environment.items()]
        lines.append(f"    環境変数: {', '.join(env)}")
    if plan is not None:
        lv = plan.levels.get(name)
        lines.append(f"    起動レベル: {'CYCLE' if lv == U32_MAX else lv}")
        if name in plan.candidates:  # stage 2: how many servers could take it on the pristine table
            cnt, first = plan.candidates[name]
            lines.append(f"    配置候補: {cnt} 台" + (f" (最初: {first})" if first else ""))
        if name in plan.assignment:
            lines.append(f"    配置先: {plan.assignment[name]}")
        elif name in plan.rejected:
            lines.append(f"    配置先: (配置不可: {plan.rejected[name]})")
        else:
            lines.append("    配置先: local")
    return lines


_FOOTER = "[dry-run] 実際の操作は行われません。--dry-run を外して実行してください。"


def format_up_dry_run(flow: Flow, stage_name: str, plan: Plan | None = None) -> str:
    """up.rs:57-136 (``print_dry_run_plan``) over ``stage.services``."""
    stage = flow.stages[stage_name]
    lines = [f"[dry-run] ステージ '{stage_name}' の起動計画:", "",
             f"  ネットワーク: {get_network_name(flow.name, stage_name)} (作成予定)"]
    for name in stage.services:
        lines += _service_block(flow, stage_name, name, "", plan)
    lines += ["", _FOOTER]
    return "\n".join(lines) + "\n"


def format_deploy_dry_run(flow: Flow, stage_name: str, target_services: list[str], tenant_line: str,
                          plan: Plan | None = None) -> str:
    """deploy.rs:14-100 (``print_dry_run_plan``) over the filtered target
    services; ``tenant_line`` is the already-resolved tenant description
    (deploy.rs:475-485)."""
    lines = [f"[dry-run] ステージ '{stage_name}' のデプロイ計画:", "", f"  テナント: {tenant_line}", "",
             f"  ネットワーク: {get_network_name(flow.name, stage_name)} (作成予定)"]
    for name in target_services:
        lines += _service_block(flow, stage_name, name, " (停止・削除→再作成)", plan)
    lines += ["", _FOOTER]
    return "\n".join(lines) + "\n"


# ---- ordering consumers -------------------------------------

def start_waves(plan: Plan) -> list[list[str]]:
    """Parallel start waves for ``DeployEngine::create_and_start``
    (crates/fleetflow-container/src/engine.rs:355-452 starts services one by one in
    ``order_by_dependencies`` order).  Wave k holds the stage's services at level k
    in declaration order; every dependency of a wave-k service is in an earlier
    wave, so a wave's containers may be created and started concurrently (one
    ``join_all`` per wave).  Levels that no service has are skipped.  CYCLE
    services (level U32_MAX) are in no wave: the reference would start them in
    bucket 2 (engine.rs:83); the plan reports them in ``plan.rejected``."""
    by_level: dict[int, list[str]] = {}
    seen = set()
    for name in plan.level_order:
        lv = plan.levels[name]
        if lv == U32_MAX or name in seen:
            continue
        seen.add(name)
        by_level.setdefault(lv, []).append(name)
    return [by_level[k] for k in sorted(by_level)]


def unit_base_name(project: str, stage: str, service: str) -> str:
    """crates/fleetflow-container/src/quadlet.rs ``unit_base_name``: ``{project}-{stage}-{service}``."""
    return f"{project}-{stage}-{service}"


def quadlet_ordering_lines(project: str, stage: str, depends_on: list[str]) -> list[str]:
    """``[Unit]`` ordering of a generated ``.container`` unit, as the reference emits
    it (crates/fleetflow-container/src/quadlet.rs:95-100): for each dependency, in
    ``depends_on`` order, ``After=`` and ``Requires=`` on its generated service."""
    out = []
    for dep in depends_on:
        unit = f"{unit_base_name(project, stage, dep)}.service"
        out += [f"After={unit}", f"Requires={unit}"]
    return out


def compose_depends_on_lines(depends_on: list[str]) -> list[str]:
    """``depends_on:`` block of a compose service (crates/fleetflow-container/src/compose.rs:156-162);
    names are YAML-quoted by the reference only when they need it, which service
    names never do."""
    if not depends_on:
        return []
    return ["    depends_on:"] + [f"      - {d}" for d in depends_on]


def wave_start_script(plan: Plan, project: str) -> list[str]:
    """Human-readable start schedule: one line per wave with its containers
    (``{project}-{stage}-{service}``, up.rs:79 naming)."""
    return [f"  wave {i}: " + ", ".join(f"{project}-{plan.stage}-{s}" for s in wave)
            for i, wave in enumerate(start_waves(plan))]
