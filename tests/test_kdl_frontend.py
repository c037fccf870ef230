"""KDL front end (fleetflow_amd/kdl.py, parser.py) and registry ingestion
(registry.py) on CPU: the reference's own parser tests, transcribed as data in
tests/golden/kdl_parser_cases.json, the two example projects BASELINE config 1
names, and KDL grammar edge cases."""
import json
import os
import random

import pytest

from fleetflow_amd import kdl
from fleetflow_amd.parser import (FlowError, determine_stage_name, extract_variables, filter_services,
                                  parse_kdl_file, parse_kdl_string, parse_kdl_string_with_stage)
from fleetflow_amd.registry import node_table, parse_plan, pool_required_labels, server_from_row

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "kdl_parser_cases.json"), encoding="utf-8"))


def _check_service(svc, exp):
    for k, v in exp.items():
        if k == "ports":
            assert [[p.host, p.container, p.protocol] for p in svc.ports] == v
        elif k == "volumes":
            assert [[x.host, x.container, x.read_only] for x in svc.volumes] == v
        elif k == "host_ip":
            assert svc.ports[0].host_ip == v
        elif k == "n_ports":
            assert len(svc.ports) == v
        elif k == "n_env":
            assert len(svc.environment) == v
        else:
            assert getattr(svc, k) == v, k


def _check_flow(flow, exp):
    if "n_services" in exp:
        assert len(flow.services) == exp["n_services"]
    if "n_stages" in exp:
        assert len(flow.stages) == exp["n_stages"]
    if "n_servers" in exp:
        assert len(flow.servers) == exp["n_servers"]
    if "name" in exp:
        assert flow.name == exp["name"]
    for name, e in exp.get("services", {}).items():
        _check_service(flow.services[name], e)
    for name, e in exp.get("stages", {}).items():
        for k, v in e.items():
            assert getattr(flow.stages[name], k) == v
    for name, e in exp.get("servers", {}).items():
        for k, v in e.items():
            assert getattr(flow.servers[name], k) == v


@pytest.mark.parametrize("case", CASES["parse"], ids=lambda c: c["source"].split()[-1])
def test_reference_parser_cases(case):
    if case["expect"].get("error"):
        with pytest.raises(FlowError):
            parse_kdl_string(case["kdl"], case.get("default_name", "test"))
        return
    _check_flow(parse_kdl_string(case["kdl"], case.get("default_name", "test")), case["expect"])


@pytest.mark.parametrize("case", CASES["include"], ids=lambda c: c["source"].split()[-1])
def test_reference_include_cases(case, tmp_path):
    for rel, text in case["files"].items():
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)
    if isinstance(case["expect"].get("error"), str):
        with pytest.raises(FlowError, match=case["expect"]["error"]):
            parse_kdl_file(tmp_path / case["main"])
        return
    _check_flow(parse_kdl_file(tmp_path / case["main"]), case["expect"])


def test_example_projects_config1():
    """BASELINE config 1 fixtures A and B (SURVEY.md 8(d) notes)."""
    a = parse_kdl_file(os.path.join(HERE, "golden", "kdl", "readme", ".fleetflow", "fleet.kdl"))
    assert a.name == ".fleetflow"  # parent directory of the file (mod.rs:43-49)
    assert a.stages["local"].services == ["postgres", "redis", "app"]
    assert a.stages["live"].services == ["postgres", "redis"]
    assert a.services["app"].depends_on == ["postgres", "redis"]
    assert a.services["postgres"].image is None and a.services["app"].image == "myapp"
    assert [p.host for p in a.services["postgres"].ports] == [11432]
    assert a.stages["local"].variables == {"APP_ENV": "development", "DEBUG": "true"}
    b = parse_kdl_file(os.path.join(HERE, "golden", "kdl", "hello-world", ".fleetflow", "fleet.kdl"))
    assert b.stages["default"].services == ["hello-oneshot", "hello-nginx"]
    assert [(p.host, p.container) for p in b.services["hello-nginx"].ports] == [(8080, 80)]
    # `read_only=true` is KDL 1 syntax; accepted through the v1 keyword fallback
    # (whether kdl 6 accepts it is unpinned)
    assert b.services["hello-nginx"].volumes[0].read_only is True
    assert determine_stage_name(None, b) == "default"


def test_stage_overrides_apply_only_with_stage():
    text = ('service "api" { image "a:1"\n depends_on "db" }\nservice "db" { image "pg" }\n'
            'stage "live" {\n service "api" {\n  image "a:2"\n  depends_on "db" "cache"\n }\n service "db"\n}\n')
    assert parse_kdl_string(text).services["api"].image == "a:1"
    f = parse_kdl_string_with_stage(text, "t", "live")
    assert f.services["api"].image == "a:2" and f.services["api"].depends_on == ["db", "cache"]


def test_depends_on_last_node_wins_and_strings_only():
    f = parse_kdl_string('service "a" {\n depends_on "x" "y"\n depends_on "z" 5 #null\n}\n')
    assert f.services["a"].depends_on == ["z"]


def test_resource_extension_nodes():
    text = ('service "api" {\n resources cpu=1500 memory=2048\n require "region=tokyo" "arch=amd64"\n'
            ' anti_affinity "web"\n ports { port host=8080 container=80 }\n}\n'
            'server "s1" {\n plan "2core-4gb"\n label "region=tokyo"\n}\n'
            'server "s2" {\n capacity cpu=8000 memory=16384\n scheduling "cordon"\n}\n'
            'server "s3" {\n provider "sakura-cloud"\n}\n')
    f = parse_kdl_string(text)
    api = f.services["api"]
    assert (api.cpu_m, api.mem_mib, api.labels, api.anti_affinity, api.host_ports) == (
        1500, 2048, ["region=tokyo", "arch=amd64"], "web", [8080])
    assert (f.servers["s1"].cpu_m, f.servers["s1"].mem_mib, f.servers["s1"].labels) == (2000, 4096, ["region=tokyo"])
    assert (f.servers["s2"].cpu_m, f.servers["s2"].schedulable) == (8000, False)
    assert f.servers["s3"].cpu_m == 0xFFFFFFFF
    with pytest.raises(FlowError):
        parse_kdl_string('service "a" { resources cpu="lots" }')


def test_variables_stage_scoping_and_errors(monkeypatch):
    text = ('variables {\n tag "1"\n}\nstage "live" {\n variables {\n tag "2"\n }\n}\n'
            'service "a" { image "x:{{ tag }}" }\n')
    assert extract_variables(text) == {"tag": "1"}
    assert extract_variables(text, "live") == {"tag": "2"}
    assert parse_kdl_string(text).services["a"].image == "x:1"
    monkeypatch.setenv("FLEET_REGION", "osaka")
    t2 = 'variables {\n a "b"\n}\nservice "s" { image "{{ FLEET_REGION }}/{{ a }}" }\n'
    assert parse_kdl_string(t2).services["s"].image == "osaka/b"
    with pytest.raises(FlowError):
        parse_kdl_string('variables {\n a "b"\n}\nservice "s" { image "{{ missing }}" }\n')


def test_filter_services_keeps_stage_order():
    assert filter_services(["a", "b", "c"], ["c", "a"], "s") == ["a", "c"]
    assert filter_services(["a", "b"], [], "s") == ["a", "b"]
    with pytest.raises(FlowError):
        filter_services(["a"], ["z"], "s")


# ---- KDL grammar ------------------------------------------------------------------------------
def test_kdl_grammar_edge_cases():
    doc = kdl.parse(r'''
// line comment
/* block /* nested */ comment */
node1 1 -2 +3 0x1F 0o17 0b101 1_000 1.5 -2.5e3 #true #false #null #inf "s\n\"q\"\u{41}" bare
/-skipped node { with children }
node2 /-skipped-arg kept key=1 key=2 /-other=3 (type)"typed" ; node3
node4 {
    child a=#"raw "quoted" string"# b=r"v1 raw"
    /-gone
}
node5 \
    continued
"quoted name" x
multi """
    line one
      line two
    """
''')
    names = [n.name for n in doc]
    assert names == ["node1", "node2", "node3", "node4", "node5", "quoted name", "multi"]
    a = doc[0].args()
    assert a[:8] == [1, -2, 3, 31, 15, 5, 1000, 1.5]
    assert a[8] == -2500.0 and a[9] is True and a[10] is False and a[11] is None and a[12] == float("inf")
    assert a[13] == 's\n"q"A' and a[14] == "bare"
    assert doc[1].args() == ["kept", "typed"] and doc[1].get("key") == 2 and not doc[1].has("other")
    ch = doc[3].children
    assert len(ch) == 1 and ch[0].get("a") == 'raw "quoted" string' and ch[0].get("b") == "v1 raw"
    assert doc[4].args() == ["continued"]
    assert doc[6].args() == ["line one\n  line two"]
    assert kdl.parse("") == [] and kdl.parse("a {}\n")[0].children == []


@pytest.mark.parametrize("bad", ['node "unterminated', "node {", "}", "a=1", 'node #bogus', 'n "a"{}x',
                                 "/* open", 'n "bad \\q"'])
def test_kdl_errors(bad):
    with pytest.raises(kdl.KdlError):
        kdl.parse(bad)


def test_kdl_dumps_roundtrip():
    src = 'a 1 "two" k=#true {\n    b "x\\ny" #null\n}\nc\n'
    doc = kdl.parse(src)
    assert kdl.parse(kdl.dumps(doc)) == doc


# ---- registry ingestion --------------------------------------------------------------------------
def test_parse_plan_known_answers(kats):
    for case in kats["parse_plan"]:
        assert list(parse_plan(case["plan"])) == case["expected"], case["source"]


def test_parse_plan_matches_oracle_on_random_strings(P):
    rng = random.Random(7)
    alphabet = "0123456789-+coregbx "
    for _ in range(3000):
        s = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 12)))
        assert parse_plan(s) == P.parse_plan(s), s
    for s in ["99999999999core-1gb", "-3core-2gb", "2corecore-4gbgb", "2core-4", "core-gb", "+7core-+8gb"]:
        assert parse_plan(s) == P.parse_plan(s), s


def test_server_rows_to_node_table():
    rows = [
        {"slug": "web-02", "capacity": {"cpu_cores": 8, "memory_gb": 16}, "allocated": {"cpu_cores": 2,
         "memory_gb": 4}, "labels": {"tier": "pro", "region": "tokyo", "extras": {"gpu": "mi355x"}}},
        {"slug": "web-01", "plan": "4core-8gb", "scheduling": "cordon"},
        {"slug": "old", "capacity": {"cpu_cores": 1, "memory_gb": 1}, "deleted_at": "2026-01-01T00:00:00Z"},
        {"slug": "db-01", "capacity": {"cpu_cores": 2, "memory_gb": 4}, "allocated": {"cpu_cores": 3}},
        {"slug": "bare"},
    ]
    t = node_table(rows)
    assert [s.slug for s in t] == ["bare", "db-01", "web-01", "web-02"]  # ORDER BY slug, live only
    bare, db, w1, w2 = t
    assert (bare.cpu_m, bare.mem_mib, bare.schedulable) == (0xFFFFFFFF, 0xFFFFFFFF, True)
    assert (db.cpu_m, db.mem_mib) == (0, 4096)  # over-allocated clamps at 0
    assert (w1.cpu_m, w1.mem_mib, w1.schedulable) == (4000, 8192, False)
    assert (w2.cpu_m, w2.mem_mib) == (6000, 12288)
    assert w2.labels == ["tier=pro", "region=tokyo", "gpu=mi355x"]
    assert server_from_row({"slug": "d", "scheduling": "drain"}).schedulable is False
    assert pool_required_labels({"required_labels": {"tier": "pro", "arch": "amd64"}}) == ["arch=amd64", "tier=pro"]
