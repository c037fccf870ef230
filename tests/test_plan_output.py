"""Plan output (fleetflow_amd/plan_output.py) on CPU: the dry-run text of
up.rs:57-136 / deploy.rs:14-100 for BASELINE config 1's fixtures, and the JSON
plan round trip.  The GPU-computed plan for the same fixtures is checked in
tests/test_gpu_parity.py::test_dry_run_from_kdl."""
import json
import os

from fleetflow_amd.flow import U32_MAX, Plan
from fleetflow_amd.parser import parse_kdl_file, parse_kdl_string
from fleetflow_amd.plan_output import (format_deploy_dry_run, format_up_dry_run, is_sensitive_key, plan_from_json,
                                       plan_to_json)

HERE = os.path.dirname(os.path.abspath(__file__))
FIX_A = os.path.join(HERE, "golden", "kdl", "readme", ".fleetflow", "fleet.kdl")


def test_up_dry_run_fixture_a_matches_reference_layout():
    flow = parse_kdl_file(FIX_A)
    flow.name = "readme"
    text = format_up_dry_run(flow, "local")
    lines = text.splitlines()
    assert lines[0] == "[dry-run] ステージ 'local' の起動計画:"
    assert lines[2] == "  ネットワーク: readme-local (作成予定)"
    blocks = text.split("\n\n")[2:-1]
    assert [b.splitlines()[0] for b in blocks] == ["  サービス: postgres", "  サービス: redis", "  サービス: app"]
    pg = blocks[0].splitlines()
    assert pg[1:5] == ["    コンテナ: readme-local-postgres", "    イメージ: (未設定)", "    ポート: 11432 → 5432/tcp",
                       "    ボリューム: ./data/postgres → /var/lib/postgresql/data (rw)"]
    env = pg[5].removeprefix("    環境変数: ").split(", ")
    assert sorted(env) == ["POSTGRES_DB=flowdb", "POSTGRES_PASSWORD=***", "POSTGRES_USER=flowuser"]
    app = blocks[2].splitlines()
    assert app[2] == "    イメージ: myapp"
    assert lines[-1] == "[dry-run] 実際の操作は行われません。--dry-run を外して実行してください。"


def test_deploy_dry_run_with_plan_lines():
    flow = parse_kdl_string('service "a" { image "x" }\nservice "b" {\n depends_on "a"\n}\n'
                            'stage "s" {\n service "a"\n service "b"\n server "vps-01"\n}\n', "proj")
    plan = Plan("s", ["a", "b"], {"a": 0, "b": 1}, ["a", "b"], {"a": "vps-01"}, {"b": "NOFIT"})
    text = format_deploy_dry_run(flow, "s", ["a", "b"], "acme (CLI flag --tenant)", plan)
    lines = text.splitlines()
    assert lines[2] == "  テナント: acme (CLI flag --tenant)"
    assert "    コンテナ: proj-s-a (停止・削除→再作成)" in lines
    assert lines[lines.index("  サービス: a") + 3:lines.index("  サービス: a") + 5] == ["    起動レベル: 0",
                                                                                   "    配置先: vps-01"]
    assert "    配置先: (配置不可: NOFIT)" in lines


def test_plan_json_roundtrip():
    plan = Plan("s", ["a", "b", "c"], {"a": 0, "b": U32_MAX, "c": 1}, ["a", "c", "b"], {"a": "n1"},
                {"b": "CYCLE", "c": "NOFIT"})
    d = json.loads(plan_to_json(plan))
    assert d["levels"] == {"a": 0, "b": None, "c": 1}
    assert plan_from_json(plan_to_json(plan)) == plan


def test_sensitive_keys():
    assert [is_sensitive_key(k) for k in ["DB_PASSWORD", "api_key", "TOKEN", "SECRET_X", "USER"]] == [
        True, True, True, True, False]


# ---- ordering consumers ----------------------------------------
def test_start_waves_group_levels_in_declaration_order():
    from fleetflow_amd.plan_output import start_waves, wave_start_script
    # README fixture shape: postgres, redis (level 0) then app (level 1); a cycle pair is left out
    plan = Plan("local", ["postgres", "redis", "app", "x", "y"],
                {"postgres": 0, "redis": 0, "app": 1, "x": U32_MAX, "y": U32_MAX},
                ["postgres", "redis", "app", "x", "y"], {}, {"x": "CYCLE", "y": "CYCLE"})
    assert start_waves(plan) == [["postgres", "redis"], ["app"]]
    assert wave_start_script(plan, "readme") == ["  wave 0: readme-local-postgres, readme-local-redis",
                                                 "  wave 1: readme-local-app"]
    # a level with no service (deps outside the stage put a root at level 1) is skipped
    plan2 = Plan("s", ["b", "a"], {"a": 1, "b": 3}, ["a", "b"], {}, {})
    assert start_waves(plan2) == [["a"], ["b"]]


def test_start_waves_respect_every_dependency():
    """Every depends_on edge inside the stage goes from an earlier wave to a later one."""
    import numpy as np
    from oracle import pyoracle as P
    from fleetflow_amd.plan_output import start_waves
    rng = np.random.default_rng(3)
    names = [f"s{i}" for i in range(60)]
    deps = {n: [names[j] for j in rng.integers(0, i, rng.integers(0, 3))] if i else [] for i, n in enumerate(names)}
    # levels from the pure-Python oracle twin over the reversed CSR
    V = len(names)
    idx = {n: i for i, n in enumerate(names)}
    rows = [[] for _ in range(V)]
    for n in names:
        for d in deps[n]:
            rows[idx[d]].append(idx[n])
    row_ptr = [0]
    col = []
    for r in rows:
        col += r
        row_ptr.append(len(col))
    has_deps = [1 if deps[n] else 0 for n in names]
    level, order = P.levelize(V, row_ptr, col, has_deps)
    plan = Plan("s", names, {n: int(level[i]) for i, n in enumerate(names)},
                [names[i] for i in order], {}, {})
    wave_of = {n: w for w, wave in enumerate(start_waves(plan)) for n in wave}
    assert sorted(wave_of) == sorted(names)
    for n in names:
        for d in deps[n]:
            assert wave_of[d] < wave_of[n]


def test_quadlet_and_compose_ordering_match_reference_emitters():
    """quadlet.rs:529-540 (After=/Requires= per dependency) and compose.rs:156-162."""
    from fleetflow_amd.plan_output import compose_depends_on_lines, quadlet_ordering_lines
    lines = quadlet_ordering_lines("myapp", "live", ["db", "redis"])
    assert lines == ["After=myapp-live-db.service", "Requires=myapp-live-db.service",
                     "After=myapp-live-redis.service", "Requires=myapp-live-redis.service"]
    assert quadlet_ordering_lines("myapp", "live", []) == []
    assert compose_depends_on_lines(["db"]) == ["    depends_on:", "      - db"]
    assert compose_depends_on_lines([]) == []
