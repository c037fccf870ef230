"""KDL front end: ``fleet.kdl`` text -> ``Flow``.

This mirrors crates/fleetflow-core/src/parser/ (mod.rs, service.rs, stage.rs,
port.rs, volume.rs, cloud.rs) for the fields the plan path reads. The
resource-request extension of SPEC.md 4 rides on child nodes that the
reference parser skips (``_ => {}`` at parser/service.rs:222), so a file
written for the planner still parses unchanged upstream.

Function names match the reference: ``parse_kdl_string``,
``parse_kdl_string_with_stage``, ``parse_kdl_file``, ``parse_service``,
``parse_stage``, ``parse_server``, ``parse_port``, ``parse_volume``,
``extract_variables``.
"""
from __future__ import annotations

import glob as _glob
import os
import re

from . import kdl
from .flow import U32_MAX, Flow, Port, Server, Service, Stage, Volume
from .kdl import as_int, as_str


class FlowError(ValueError):
    """fleetflow_core::FlowError (error.rs) for the parse path."""


_RESTART = {"no", "always", "on-failure", "unless-stopped"}


def _first_str(node):
    return as_str(node.first())


def _u32(v, what):
    if not kdl.is_int(v) or not 0 <= v <= U32_MAX:
        raise FlowError(f"{what} must be an integer in 0..{U32_MAX}, got {v!r}")
    return v


# ---- parser/port.rs:11-61 ----------------------------------------------------------------
def parse_port(node) -> Port | None:
    """``port host=8080 container=3000`` or positional ``port 8080 3000``. Named
    properties win, then the 1st/2nd entries (container falls back to the
    1st)."""
    def u16(v):
        return v & 0xFFFF if kdl.is_int(v) else None  # Rust `as u16` truncation

    host = u16(node.get("host")) if node.has("host") else None
    if host is None:
        host = u16(node.entries[0][1]) if node.entries else None
    if host is None:
        return None
    container = u16(node.get("container")) if node.has("container") else None
    if container is None:
        e = node.entries[1][1] if len(node.entries) > 1 else (node.entries[0][1] if node.entries else None)
        container = u16(e)
    if container is None:
        return None
    proto = as_str(node.get("protocol"))
    return Port(host, container, proto if proto in ("tcp", "udp") else "tcp", as_str(node.get("host_ip")))


# ---- parser/volume.rs:8-58 ----------------------------------------------------------------
def parse_volume(node) -> Volume | None:
    if len(node.entries) < 2:
        return None
    host, container = as_str(node.entries[0][1]), as_str(node.entries[1][1])
    if host is None or container is None:
        return None
    ro = node.get("read_only")
    read_only = ro if isinstance(ro, bool) else (ro == "true") if ro in ("true", "false") else False
    return Volume(host, container, read_only)


# ---- parser/service.rs:11-230 (+ SPEC.md 4 extension) -------------------------------------
def parse_service(node) -> tuple[str, Service]:
    name = _first_str(node)
    if name is None:
        raise FlowError("service requires a name")
    svc = Service()
    for key, v in node.entries:
        if key in ("type", "service_type"):
            svc.service_type = v.lower() if isinstance(v, str) and v.lower() in ("container", "static") else None
        elif key in ("command", "image", "version", "registry"):
            setattr(svc, key, as_str(v))
        elif key == "restart":
            svc.restart = v if v in _RESTART else None
    for ch in node.children or []:
        n = ch.name
        if n in ("image", "version", "command", "registry"):
            setattr(svc, n, _first_str(ch))
        elif n == "ports":
            for pn in ch.children or []:
                if pn.name == "port":
                    p = parse_port(pn)
                    if p is not None:
                        svc.ports.append(p)
        elif n == "port":
            p = parse_port(ch)
            if p is not None:
                svc.ports.append(p)
        elif n in ("environment", "env"):
            if ch.children is not None:
                for en in ch.children:
                    svc.environment[en.name] = _first_str(en) or ""
            else:
                val = _first_str(ch)
                if val is not None and "=" in val:
                    k, v = val.split("=", 1)
                    svc.environment[k.strip()] = v.strip()
        elif n == "volumes":
            for vn in ch.children or []:
                if vn.name == "volume":
                    vol = parse_volume(vn)
                    if vol is not None:
                        svc.volumes.append(vol)
        elif n == "depends_on":
            # last depends_on node wins; only string entries count (service.rs:124-130)
            svc.depends_on = [v for _, v in ch.entries if isinstance(v, str)]
        elif n == "restart":
            r = _first_str(ch)
            svc.restart = r if r in _RESTART else None
        # ---- SPEC.md 4: resource-request extension ----
        elif n == "resources":
            if ch.has("cpu"):
                svc.cpu_m = _u32(ch.get("cpu"), f"service {name}: resources cpu")
            if ch.has("memory"):
                svc.mem_mib = _u32(ch.get("memory"), f"service {name}: resources memory")
        elif n == "require":
            svc.labels = svc.labels + [v for _, v in ch.entries if isinstance(v, str)]
        elif n == "anti_affinity":
            svc.anti_affinity = _first_str(ch)
    return name, svc


# ---- parser/stage.rs:12-93 ----------------------------------------------------------------
def parse_stage(node) -> tuple[str, Stage, dict[str, Service]]:
    name = _first_str(node)
    if name is None:
        raise FlowError("stage requires a name")
    st = Stage()
    overrides: dict[str, Service] = {}
    for ch in node.children or []:
        if ch.name == "service":
            sn = _first_str(ch)
            if sn is not None:
                st.services.append(sn)
                if ch.children is not None:
                    overrides[sn] = parse_service(ch)[1]
        elif ch.name == "server":
            sv = _first_str(ch)
            if sv is not None:
                st.servers.append(sv)
        elif ch.name == "variables":
            for vn in ch.children or []:
                st.variables[vn.name] = _first_str(vn) or ""
        elif ch.name == "registry":
            st.registry = _first_str(ch)
        elif ch.name == "backend":
            raw = _first_str(ch)
            if raw is None:
                raise FlowError("backend requires a value (docker|quadlet|compose)")
            if raw.lower() not in ("docker", "quadlet", "compose"):
                raise FlowError(f"unknown backend '{raw}' (expected docker|quadlet|compose)")
            st.backend = raw.lower()
    return name, st, overrides


# ---- parser/cloud.rs:46-140 (+ SPEC.md 4 capacity/labels/scheduling) ------------------------
def parse_server(node) -> tuple[str, Server]:
    from .registry import parse_plan

    name = _first_str(node)
    if name is None:
        raise FlowError("server requires a name")
    srv = Server(slug=name)
    cap_cpu = cap_mem = None
    for ch in node.children or []:
        if ch.name == "provider":
            srv.provider = _first_str(ch) or ""
        elif ch.name == "plan":
            srv.plan = _first_str(ch)
        elif ch.name == "capacity":
            if ch.has("cpu"):
                cap_cpu = _u32(ch.get("cpu"), f"server {name}: capacity cpu")
            if ch.has("memory"):
                cap_mem = _u32(ch.get("memory"), f"server {name}: capacity memory")
        elif ch.name == "label":
            srv.labels = srv.labels + [v for _, v in ch.entries if isinstance(v, str)]
        elif ch.name == "scheduling":
            srv.schedulable = (_first_str(ch) or "schedulable") == "schedulable"
    if srv.plan is not None:  # provider.rs:15-30 plan string -> (cores, GB)
        cores, gb = parse_plan(srv.plan)
        srv.cpu_m = min(max(cores, 0) * 1000, U32_MAX)
        srv.mem_mib = min(max(gb, 0) * 1024, U32_MAX)
    if cap_cpu is not None:
        srv.cpu_m = cap_cpu
    if cap_mem is not None:
        srv.mem_mib = cap_mem
    return name, srv


# ---- template.rs:227-340: variables + {{ }} rendering ------------------------------------------
_STAGE_RE = re.compile(r"""stage\s+["'][^"']+["']\s*\{""", re.S)
_VARS_RE = re.compile(r"variables\s*\{(?P<content>.*?)\}", re.S)
_TMPL_RE = re.compile(r"\{\{\s*([A-Za-z_][A-Za-z0-9_]*)\s*\}\}")


def _matching_brace(text, open_pos):
    """template.rs find_matching_brace: quote-aware, backslash-escape-aware."""
    depth, pos, in_str, esc = 1, open_pos + 1, False, False
    while pos < len(text) and depth > 0:
        c = text[pos]
        if esc:
            esc = False
        elif c == "\\":
            esc = True
        elif c == '"':
            in_str = not in_str
        elif not in_str:
            depth += (c == "{") - (c == "}")
        pos += 1
    return pos - 1 if depth == 0 else None


def _vars_from(content):
    out = {}
    for m in _VARS_RE.finditer(content):
        try:
            doc = kdl.parse("extracted {\n" + m.group("content") + "\n}")
        except kdl.KdlError as e:
            raise FlowError(f"KDL parse error (variables block): {e}") from e
        for vn in doc[0].children or []:
            if vn.entries:
                out[vn.name] = vn.entries[0][1]
    return out


def extract_variables(content: str, stage: str | None = None) -> dict:
    """Global ``variables {}`` blocks (outside every stage block), then the named
    stage's blocks on top (template.rs:239-313)."""
    ranges = []
    for m in _STAGE_RE.finditer(content):
        end = _matching_brace(content, m.end() - 1)
        if end is not None:
            ranges.append((m.start(), end + 1))
    glob_text, last = [], 0
    for a, b in ranges:
        if a < last:
            continue
        glob_text.append(content[last:a])
        last = b
    glob_text.append(content[last:])
    out = _vars_from("".join(glob_text))
    if stage is not None:
        sre = re.compile(r"""stage\s+["']""" + re.escape(stage) + r"""["']\s*\{""", re.S)
        for m in sre.finditer(content):
            end = _matching_brace(content, m.end() - 1)
            if end is not None:
                out.update(_vars_from(content[m.end():end]))
    return out


def _tera_str(v):
    if v is True:
        return "true"
    if v is False:
        return "false"
    if v is None:
        return ""
    return str(v)


def render_template(content: str, variables: dict) -> str:
    """``{{ name }}`` substitution with the flow variables plus FLEET_/CI_/APP_
    environment variables (template.rs:69-95). An undefined name is an error,
    as in the reference's template engine. Other template syntax is not
    supported here and is rejected."""
    ctx = {k: _tera_str(v) for k, v in variables.items()}
    for k, v in os.environ.items():
        if k.startswith(("FLEET_", "CI_", "APP_")):
            ctx[k] = v

    def sub(m):
        k = m.group(1)
        if k not in ctx:
            raise FlowError(f"template render error: variable `{k}` not found")
        return ctx[k]

    out = _TMPL_RE.sub(sub, content)
    if "{{" in out or "{%" in out:
        raise FlowError("template render error: only {{ name }} substitutions are supported")
    return out


# ---- parser/mod.rs:139-299 --------------------------------------------------------------------
def parse_kdl_string(content: str, default_name: str = "unnamed") -> Flow:
    return parse_kdl_string_with_stage(content, default_name, None)


def parse_kdl_string_with_stage(content: str, default_name: str = "unnamed", target_stage: str | None = None) -> Flow:
    variables = extract_variables(content)
    expanded = render_template(content, variables) if variables else content
    return _parse_raw(expanded, default_name, target_stage)


def _parse_raw(content, default_name, target_stage) -> Flow:
    try:
        doc = kdl.parse(content)
    except kdl.KdlError as e:
        raise FlowError(str(e)) from e
    flow = Flow(name=default_name)
    stage_overrides: dict[str, dict[str, Service]] = {}
    for node in doc:
        n = node.name
        if n == "project":
            pn = _first_str(node)
            if pn is not None:
                flow.name = pn
        elif n == "stage":
            sn, st, ov = parse_stage(node)
            flow.stages[sn] = st
            if ov:
                stage_overrides[sn] = ov
        elif n == "service":
            name, svc = parse_service(node)
            if name in flow.services:
                flow.services[name].merge(svc)
            else:
                flow.services[name] = svc
        elif n == "server":
            name, srv = parse_server(node)
            flow.servers[name] = srv
        elif n == "variables":
            for vn in node.children or []:
                flow.variables[vn.name] = _first_str(vn) or ""
        elif n == "registry":
            r = _first_str(node)
            if r is not None:
                flow.registry = r
        # include (already expanded by parse_kdl_file), provider, tenant, unknown: skipped
    if target_stage is not None and target_stage in stage_overrides:
        for name, svc in stage_overrides[target_stage].items():
            if name in flow.services:
                flow.services[name].merge(svc)
            else:
                flow.services[name] = svc
    return flow


def _read_with_includes(path, base_dir, visited) -> str:
    """mod.rs:55-135: expand ``include "file"`` / ``include "dir/*.kdl"`` recursively,
    relative to the including file; a file seen twice is a circular include."""
    ap = path if os.path.isabs(path) else os.path.join(base_dir, path)
    try:
        ap = os.path.realpath(ap, strict=True)
    except OSError as e:
        raise FlowError(f"path resolution error: {path}: {e}") from e
    if ap in visited:
        raise FlowError(f"Circular include detected: {ap}")
    visited.add(ap)
    with open(ap, encoding="utf-8") as f:
        content = f.read()
    try:
        doc = kdl.parse(content)
    except kdl.KdlError as e:
        raise FlowError(f"KDL parse error in {ap}: {e}") from e
    cur = os.path.dirname(ap)
    out = []
    for node in doc:
        if node.name == "include":
            inc = _first_str(node)
            if inc is None:
                continue
            if "*" in inc:
                for p in sorted(_glob.glob(os.path.join(cur, inc))):
                    out.append(_read_with_includes(p, cur, visited) + "\n")
            else:
                out.append(_read_with_includes(os.path.join(cur, inc), cur, visited) + "\n")
        else:
            out.append(kdl.dumps([node]))
    return "".join(out)


def parse_kdl_file(path: str, target_stage: str | None = None) -> Flow:
    """mod.rs:31-52: includes expanded, project name defaults to the parent
    directory's name."""
    path = os.fspath(path)
    base = os.path.dirname(path) or "."
    content = _read_with_includes(path, base, set())
    name = os.path.basename(os.path.dirname(os.path.abspath(path))) or "unnamed"
    return parse_kdl_string_with_stage(content, name, target_stage)


def filter_services(stage_services: list[str], filters: list[str], stage_name: str) -> list[str]:
    """crates/fleetflow/src/utils.rs:46-73: ``-n`` filter, stage order kept."""
    if not filters:
        return list(stage_services)
    for f in filters:
        if f not in stage_services:
            raise FlowError(f"service '{f}' is not in stage '{stage_name}'. available: {', '.join(stage_services)}")
    return [s for s in stage_services if s in filters]


def determine_stage_name(stage: str | None, flow: Flow) -> str:
    """crates/fleetflow/src/utils.rs:4-25."""
    if stage is not None:
        return stage
    if "default" in flow.stages:
        return "default"
    if len(flow.stages) == 1:
        return next(iter(flow.stages))
    raise FlowError("specify a stage: available stages: " + ", ".join(flow.stages))
