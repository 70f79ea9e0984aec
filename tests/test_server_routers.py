"""REST API tests against an in-memory server (reference test strategy: ``src/tests/_internal/
server/routers/test_*.py`` — TestClient + real DB, background tasks driven explicitly)."""

import json

import pytest

from tests.conftest import ADMIN_TOKEN


def _task(name="t1", **kw):
    conf = {"type": "task", "commands": ["echo hi"]}
    conf.update(kw)
    return {"run_spec": {"run_name": name, "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                         "configuration": conf, "ssh_key_pub": ""}}


def _init_virtual_repo(client):
    r = client.post("/api/project/main/repos/init", json={"repo_id": "virt", "repo_info": {"repo_type": "virtual"}})
    assert r.status_code == 200, r.text


# ---- server / auth ----------------------------------------------------------------------------
def test_server_info(client):
    r = client.post("/api/server/get_info")
    assert r.status_code == 200
    assert r.json()["server_version"]


def test_healthcheck(client):
    assert client.get("/healthcheck").json() == {"status": "running"}


def test_requires_token(client):
    r = client.post("/api/users/get_my_user", headers={"Authorization": "Bearer nope"})
    assert r.status_code in (401, 403)
    r = client.post("/api/projects/list", headers={"Authorization": ""})
    assert r.status_code in (401, 403)


def test_incompatible_client_version(client):
    r = client.post("/api/server/get_info", headers={"X-API-VERSION": "99.0.0"})
    assert r.status_code == 400


# ---- users ------------------------------------------------------------------------------------
def test_users_crud(client):
    me = client.post("/api/users/get_my_user").json()
    assert me["username"] == "admin" and me["creds"]["token"] == ADMIN_TOKEN
    r = client.post("/api/users/create", json={"username": "alice", "global_role": "user"})
    assert r.status_code == 200, r.text
    alice_token = r.json()["creds"]["token"]
    names = {u["username"] for u in client.post("/api/users/list").json()}
    assert {"admin", "alice"} <= names
    # a non-admin only sees itself and cannot create users
    r = client.post("/api/users/list", headers={"Authorization": f"Bearer {alice_token}"})
    assert [u["username"] for u in r.json()] == ["alice"]
    r = client.post("/api/users/create", json={"username": "bob"}, headers={"Authorization": f"Bearer {alice_token}"})
    assert r.status_code == 403
    r = client.post("/api/users/refresh_token", json={"username": "alice"})
    assert r.json()["creds"]["token"] != alice_token
    client.post("/api/users/delete", json={"users": ["alice"]})
    assert "alice" not in {u["username"] for u in client.post("/api/users/list").json()}


def test_duplicate_user_rejected(client):
    assert client.post("/api/users/create", json={"username": "carol"}).status_code == 200
    r = client.post("/api/users/create", json={"username": "carol"})
    assert r.status_code == 400
    assert r.json()["detail"][0]["code"] == "resource_exists"


# ---- projects ---------------------------------------------------------------------------------
def test_projects_and_members(client):
    assert [p["project_name"] for p in client.post("/api/projects/list").json()] == ["main"]
    r = client.post("/api/projects/create", json={"project_name": "research"})
    assert r.status_code == 200, r.text
    u = client.post("/api/users/create", json={"username": "dan"}).json()
    dan = {"Authorization": f"Bearer {u['creds']['token']}"}
    assert client.post("/api/projects/research/get", headers=dan).status_code == 403
    r = client.post("/api/projects/research/set_members",
                    json={"members": [{"username": "admin", "project_role": "admin"},
                                      {"username": "dan", "project_role": "user"}]})
    assert r.status_code == 200, r.text
    assert client.post("/api/projects/research/get", headers=dan).status_code == 200
    assert [p["project_name"] for p in client.post("/api/projects/list", headers=dan).json()] == ["research"]
    # a plain member cannot manage members
    r = client.post("/api/projects/research/set_members", json={"members": []}, headers=dan)
    assert r.status_code == 403
    client.post("/api/projects/delete", json={"projects_names": ["research"]})
    assert [p["project_name"] for p in client.post("/api/projects/list").json()] == ["main"]


def test_invalid_project_name(client):
    assert client.post("/api/projects/create", json={"project_name": "bad name!"}).status_code in (400, 422)


# ---- secrets ----------------------------------------------------------------------------------
def test_secrets(client):
    r = client.post("/api/project/main/secrets/add", json={"name": "HF_TOKEN", "value": "s3cr3t"})
    assert r.status_code == 200, r.text
    assert client.post("/api/project/main/secrets/get", json={"name": "HF_TOKEN"}).json()["value"] == "s3cr3t"
    listed = client.post("/api/project/main/secrets/list").json()
    assert [s["name"] for s in listed] == ["HF_TOKEN"]
    client.post("/api/project/main/secrets/delete", json={"secrets_names": ["HF_TOKEN"]})
    assert client.post("/api/project/main/secrets/list").json() == []


# ---- repos ------------------------------------------------------------------------------------
def test_repos_and_code_upload(client):
    _init_virtual_repo(client)
    repos = client.post("/api/project/main/repos/list").json()
    assert [r["repo_id"] for r in repos] == ["virt"]
    r = client.post("/api/project/main/repos/upload_code?repo_id=virt", content=b"tar-bytes",
                    headers={"content-type": "application/octet-stream"})
    assert r.status_code == 200 and len(r.json()["blob_hash"]) == 64
    client.post("/api/project/main/repos/delete", json={"repos_ids": ["virt"]})
    assert client.post("/api/project/main/repos/list").json() == []


# ---- backends ---------------------------------------------------------------------------------
def test_backend_types(client):
    types = client.post("/api/backends/list_types").json()
    assert "local" in types and "remote" in types


# ---- runs -------------------------------------------------------------------------------------
def test_run_plan_submit_stop_delete(client):
    _init_virtual_repo(client)
    plan = client.post("/api/project/main/runs/get_plan", json=_task("r1"))
    assert plan.status_code == 200, plan.text
    body = plan.json()
    assert body["job_plans"][0]["job_spec"]["commands"][-1].endswith("echo hi")
    r = client.post("/api/project/main/runs/submit", json=_task("r1"))
    assert r.status_code == 200, r.text
    assert r.json()["status"] == "submitted"
    # duplicate active run name rejected
    assert client.post("/api/project/main/runs/submit", json=_task("r1")).status_code == 400
    runs = client.post("/api/runs/list", json={}).json()
    assert [x["run_spec"]["run_name"] for x in runs] == ["r1"]
    got = client.post("/api/project/main/runs/get", json={"run_name": "r1"}).json()
    assert got["jobs"][0]["job_submissions"][0]["status"] == "submitted"
    assert client.post("/api/project/main/runs/stop", json={"runs_names": ["r1"], "abort": True}).status_code == 200
    got = client.post("/api/project/main/runs/get", json={"run_name": "r1"}).json()
    assert got["status"] == "terminating"
    # cannot delete an active run
    assert client.post("/api/project/main/runs/delete", json={"runs_names": ["r1"]}).status_code == 400


def test_run_generated_name(client):
    _init_virtual_repo(client)
    r = client.post("/api/project/main/runs/submit", json=_task(None))
    assert r.status_code == 200, r.text
    assert r.json()["run_spec"]["run_name"]


def test_invalid_configuration_rejected(client):
    _init_virtual_repo(client)
    spec = _task("bad")
    spec["run_spec"]["configuration"]["unknown_field"] = 1
    assert client.post("/api/project/main/runs/submit", json=spec).status_code == 422


def test_multinode_task_creates_jobs(client):
    _init_virtual_repo(client)
    r = client.post("/api/project/main/runs/submit", json=_task("mn", nodes=2))
    assert r.status_code == 200, r.text
    jobs = r.json()["jobs"]
    assert sorted(j["job_spec"]["job_num"] for j in jobs) == [0, 1]
    assert all(j["job_spec"]["jobs_per_replica"] == 2 for j in jobs)


def test_service_replicas(client):
    _init_virtual_repo(client)
    conf = {"type": "service", "commands": ["python -m http.server 8000"], "port": 8000, "replicas": 2}
    spec = {"run_spec": {"run_name": "svc", "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                         "configuration": conf, "ssh_key_pub": ""}}
    r = client.post("/api/project/main/runs/submit", json=spec)
    assert r.status_code == 200, r.text
    assert sorted(j["job_spec"]["replica_num"] for j in r.json()["jobs"]) == [0, 1]


# ---- fleets / instances / volumes / gateways ---------------------------------------------------
def test_ssh_fleet_create_and_delete(client):
    key = {"public": "ssh-ed25519 AAAA", "private": "-----BEGIN OPENSSH PRIVATE KEY-----\nx\n"
                                                   "-----END OPENSSH PRIVATE KEY-----\n"}
    spec = {"spec": {"configuration": {"type": "fleet", "name": "onprem",
                                       "ssh_config": {"user": "ubuntu", "ssh_key": key,
                                                      "hosts": ["10.0.0.1", "10.0.0.2"]}},
                     "profile": {"name": "default"}}}
    r = client.post("/api/project/main/fleets/get_plan", json=spec)
    assert r.status_code == 200, r.text
    r = client.post("/api/project/main/fleets/create", json=spec)
    assert r.status_code == 200, r.text
    fleet = r.json()
    assert fleet["name"] == "onprem" and len(fleet["instances"]) == 2
    names = [f["name"] for f in client.post("/api/project/main/fleets/list").json()]
    assert names == ["onprem"]
    inst = client.post("/api/instances/list", json={}).json()
    assert len(inst) == 2
    assert client.post("/api/project/main/fleets/delete", json={"names": ["onprem"]}).status_code == 200


def test_volumes_list_empty(client):
    assert client.post("/api/project/main/volumes/list").json() == []
    assert client.post("/api/volumes/list", json={}).json() == []


def test_gateways_list_empty(client):
    assert client.post("/api/project/main/gateways/list").json() == []


def test_pool_list(client):
    r = client.post("/api/project/main/pool/list")
    assert r.status_code == 200


def test_logs_poll_unknown_submission(client):
    import uuid

    r = client.post("/api/project/main/logs/poll", json={"run_name": "nope", "job_submission_id": str(uuid.uuid4())})
    assert r.status_code == 200
    assert r.json()["logs"] == []


@pytest.mark.parametrize("path", ["/api/project/nope/runs/get", "/api/project/nope/fleets/list"])
def test_unknown_project(client, path):
    assert client.post(path, json={"run_name": "x"}).status_code in (403, 404, 400)


def _ui_text(client):
    """index.html plus every script module it loads."""
    import re

    html = client.get("/").text
    mods = re.findall(r'<script src="(/ui/js/[a-z]+\.js)"', html)
    assert mods, "no UI modules referenced"
    parts = [html]
    for m in mods:
        r = client.get(m)
        assert r.status_code == 200 and r.headers["content-type"].startswith("text/javascript"), m
        parts.append(r.text)
    return "\n".join(parts)


def test_web_ui_served(client):
    r = client.get("/")
    assert r.status_code == 200 and "dstack-amd" in r.text
    assert client.get("/ui/js/../../app.py").status_code == 404  # only the shipped modules
    text = _ui_text(client)
    assert "/api/runs/list" in text
    # management views over the same API: instances, members editor, backends from YAML, metrics charts
    for needle in ("/api/instances/list", "set_members", "backends/${x}", "create_yaml", "metrics/job/", "prev_run_id",
                   "fleets/delete_instances", "users/refresh_token", "form_schema", "config_values", "descending: true",
                   "fleet_ids", "job_submissions",
                   # overview, SSH-fleet form, project gateways / CLI tabs, member suggestions
                   "home()", "newfleet()", 'P("fleets/get_plan")', 'P("fleets/create")', "dstack config --url",
                   'G("set_default")', "known-users",
                   # bulk run / fleet actions, a run's jobs tab, the signed-in user's account page
                   '"runs/stop"', '"runs/delete"', "runs_names: picked()", "fleets/delete\"), { names: picked()", "jobs(r)",
                   "account()", '"/api/users/get_my_user"'):
        assert needle in text, needle


def test_web_ui_calls_only_existing_routes(client):
    """Every REST path the UI modules call is a route of the app (project-scoped ``P("...")``
    paths under ``/api/project/{project_name}/``)."""
    import re

    text = _ui_text(client)
    routes = set(client.get("/api/openapi.json").json()["paths"])
    called = set(re.findall(r'P\(["`]([a-z_]+/[a-z_]+)', text)) - {"metrics/job"}  # GET .../metrics/job/{run_name}
    assert "/api/project/{project_name}/metrics/job/{run_name}" in routes
    missing = [c for c in called if f"/api/project/{{project_name}}/{c}" not in routes]
    assert called and not missing, missing
    absolute = set(re.findall(r'api\(["`](/api/[a-z_/]+)["`]', text))
    missing = [c for c in absolute if c not in routes]
    assert absolute and not missing, missing


def test_web_ui_apply_and_offers_request_shapes(client):
    """The UI's apply / offers / fleet pages: YAML -> configurations/parse -> get_plan -> apply with
    exactly the payloads index.html builds."""
    html = _ui_text(client)
    for needle in ("configurations/parse", "runs/get_plan", "runs/apply", "fleets/get_plan", "fleets/get",
                   "spot_policy", "bytes_per_s"):
        assert needle in html, needle
    P = "/api/project/main"
    r = client.post(f"{P}/configurations/parse", json={"yaml": "type: task\nname: ui-run\ncommands: [echo hi]\n"})
    assert r.status_code == 200, r.text
    conf = r.json()["configuration"]
    assert r.json()["type"] == "task" and conf["commands"] == ["echo hi"]
    run_spec = {"run_name": conf.get("name"), "repo_id": "ui", "repo_data": {"repo_type": "virtual"},
                "configuration": conf, "ssh_key_pub": ""}
    plan = client.post(f"{P}/runs/get_plan", json={"run_spec": run_spec, "max_offers": 50})
    assert plan.status_code == 200, plan.text
    plan = plan.json()
    assert plan["job_plans"] and "total_offers" in plan["job_plans"][0]
    r = client.post(f"{P}/runs/apply", json={"plan": {"run_spec": plan["run_spec"],
                                                       "current_resource": plan["current_resource"]}, "force": False})
    assert r.status_code == 200, r.text
    assert r.json()["run_spec"]["run_name"] == "ui-run"
    # offers page: a task with gpu / spot policy / max price
    offers_conf = {"type": "task", "commands": [":"], "spot_policy": "auto", "resources": {"gpu": "MI355X:8"},
                   "max_price": 100}
    r = client.post(f"{P}/runs/get_plan", json={"run_spec": {"repo_id": "ui", "repo_data": {"repo_type": "virtual"},
                                                             "configuration": offers_conf, "ssh_key_pub": ""},
                                                "max_offers": 200})
    assert r.status_code == 200, r.text
    # fleet plan from parsed YAML
    r = client.post(f"{P}/configurations/parse", json={"yaml": "type: fleet\nname: f1\nnodes: 1\n"})
    assert r.status_code == 200, r.text
    r = client.post(f"{P}/fleets/get_plan", json={"spec": {"configuration": r.json()["configuration"]}})
    assert r.status_code == 200, r.text and "offers" in r.json()
    # bad YAML / bad configuration -> 400 with the reason
    r = client.post(f"{P}/configurations/parse", json={"yaml": "type: task\n  bad: [\n"})
    assert r.status_code == 400 and "invalid YAML" in r.json()["detail"][0]["msg"]
    r = client.post(f"{P}/configurations/parse", json={"yaml": "type: nonsense\n"})
    assert r.status_code == 400


def _form_yaml(kind, vals):
    """YAML the UI's configuration forms produce (forms.js buildConfiguration + core.js yamlish), run
    under node with the browser globals stubbed."""
    import json
    import os
    import shutil
    import subprocess

    node = shutil.which("node")
    if node is None:
        pytest.skip("node is not installed")
    major = int(subprocess.run([node, "--version"], capture_output=True, text=True).stdout.strip().lstrip("v").split(".")[0])
    if major < 12:
        pytest.skip(f"node {major} is too old")
    # node 12-15 (this image ships 12): ?? and ?. behind V8 flags; the one ??= of core.js spelled out
    # and Array.prototype.at polyfilled -- what browsers run natively
    flags = ["--harmony-nullish", "--harmony-optional-chaining"] if major < 16 else []
    ui = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dstack_amd", "server", "ui", "js")
    src = {m: open(os.path.join(ui, m)).read().replace("o[k] ??= {}", "(o[k] = o[k] ?? {})") for m in ("core.js", "forms.js")}
    script = (
        "const vm = require('vm');"
        "if (!Array.prototype.at) Array.prototype.at = function (i) { return this[i < 0 ? this.length + i : i]; };"
        "globalThis.localStorage = {getItem: () => null, setItem() {}};"
        "globalThis.document = {querySelector: () => null, querySelectorAll: () => []};"
        f"vm.runInThisContext({json.dumps(src['core.js'])});"
        f"vm.runInThisContext({json.dumps(src['forms.js'])});"
        f"process.stdout.write(vm.runInThisContext('yamlish(buildConfiguration(' + JSON.stringify({json.dumps(kind)}) + ', ' + "
        f"JSON.stringify({json.dumps(vals)}) + ')).trimStart()'));"
    )
    return subprocess.run([node, *flags, "-e", script], check=True, capture_output=True, text=True, timeout=60).stdout


def test_web_ui_forms_produce_configurations_the_server_accepts(client):
    """forms.js: each kind's form values -> YAML that configurations/parse accepts with the intended
    fields, and (runs, fleets) a plan from it."""
    P = "/api/project/main"
    cases = {
        "task": ({"name": "form-task", "commands": ["echo 1", "python -c 'print(2)'"], "gpu": "MI355X:8", "nodes": 2,
                  "env": ["HF_TOKEN", "NCCL_DEBUG=INFO"], "max_duration": "72h", "spot_policy": "auto"},
                 {"nodes": 2, "commands": ["echo 1", "python -c 'print(2)'"]}),
        "service": ({"name": "form-svc", "commands": ["vllm serve m --port 8000"], "port": 8000, "gpu": "MI355X:8",
                     "replicas": "1..4", "scaling_metric": "rps", "scaling_target": 10.0, "model": "meta-llama/Meta-Llama-3-70B"},
                    {"port": 8000}),
        "dev-environment": ({"name": "form-dev", "ide": "vscode", "gpu": "MI355X:1", "init": ["pip install x"]}, {"ide": "vscode"}),
        "fleet": ({"name": "form-fleet", "nodes": "0..4", "gpu": "MI355X:8", "placement": "cluster", "idle_duration": "30m"},
                  {"placement": "cluster"}),
        "volume": ({"name": "form-vol", "backend": "aws", "region": "us-east-1", "size": "500GB"}, {"region": "us-east-1"}),
    }
    for kind, (vals, expect) in cases.items():
        text = _form_yaml(kind, vals)
        r = client.post(f"{P}/configurations/parse", json={"yaml": text})
        assert r.status_code == 200, (kind, text, r.text)
        conf = r.json()["configuration"]
        assert r.json()["type"] == kind and conf["name"] == vals["name"], (kind, conf)
        for k, v in expect.items():
            got = conf[k]
            assert got == v or (isinstance(got, dict) and got.get("container_port") == v), (kind, k, got)
        if kind in ("task", "service", "dev-environment"):
            assert "MI355X" in json.dumps(conf["resources"]), conf["resources"]
            run_spec = {"run_name": conf["name"], "repo_id": "ui", "repo_data": {"repo_type": "virtual"},
                        "configuration": conf, "ssh_key_pub": ""}
            r = client.post(f"{P}/runs/get_plan", json={"run_spec": run_spec, "max_offers": 5})
            assert r.status_code == 200, (kind, r.text)
        elif kind == "fleet":
            assert conf["nodes"]["min"] == 0 and conf["nodes"]["max"] == 4, conf["nodes"]
            r = client.post(f"{P}/fleets/get_plan", json={"spec": {"configuration": conf}})
            assert r.status_code == 200, r.text


def test_prometheus_metrics(client):
    _init_virtual_repo(client)
    client.post("/api/project/main/runs/submit", json=_task("prom1"))
    r = client.get("/metrics")
    assert r.status_code == 200
    assert 'dstack_runs{project="main",status="submitted"} 1' in r.text
    assert "# TYPE dstack_job_gpu_util_percent gauge" in r.text


# ---- legacy pool API (reference routers/pools.py, routers/runs.py:183-219, deprecated) ----------
def test_legacy_pools_crud(client):
    r = client.post("/api/project/main/pool/create", json={"name": "p2"})
    assert r.status_code == 200, r.text
    assert client.post("/api/project/main/pool/create", json={"name": "p2"}).status_code == 400
    names = {p["name"] for p in client.post("/api/project/main/pool/list").json()}
    assert "p2" in names
    assert client.post("/api/project/main/pool/set_default", json={"pool_name": "p2"}).status_code == 200
    pools = {p["name"]: p for p in client.post("/api/project/main/pool/list").json()}
    assert pools["p2"]["default"] is True
    assert client.post("/api/project/main/pool/set_default", json={"pool_name": "nope"}).status_code == 400
    r = client.post("/api/project/main/pool/add_remote", json={
        "pool_name": "p2", "host": "10.0.0.7", "port": 22, "ssh_user": "ubuntu",
        "ssh_keys": [{"public": "ssh-ed25519 AAAA", "private": "-----BEGIN KEY-----"}],
        "instance_network": "10.0.0.0/24"})
    assert r.status_code == 200, r.text
    inst = r.json()
    assert inst["status"] == "pending" and inst["backend"] == "remote"
    # idempotent per host/port/user
    again = client.post("/api/project/main/pool/add_remote", json={
        "pool_name": "p2", "host": "10.0.0.7", "port": 22, "ssh_user": "ubuntu",
        "ssh_keys": [{"public": "ssh-ed25519 AAAA"}]}).json()
    assert again["id"] == inst["id"]
    shown = client.post("/api/project/main/pool/show", json={"name": "p2"}).json()
    assert [i["name"] for i in shown["instances"]] == [inst["name"]]
    # a pool with live instances cannot be deleted; remove the instance first
    assert client.post("/api/project/main/pool/delete", json={"name": "p2"}).status_code == 400
    r = client.post("/api/project/main/pool/remove", json={"pool_name": "p2", "instance_name": inst["name"]})
    assert r.status_code == 200, r.text
    shown = client.post("/api/project/main/pool/show", json={"name": "p2"}).json()
    assert shown["instances"][0]["status"] == "terminating"
    bad = client.post("/api/project/main/pool/add_remote", json={"host": " ", "ssh_user": "u", "ssh_keys": []})
    assert bad.status_code == 400


def test_legacy_get_offers(client):
    r = client.post("/api/project/main/runs/get_offers", json={
        "profile": {"name": "default"}, "requirements": {"resources": {"cpu": "1..", "memory": "0.1GB.."}}})
    assert r.status_code == 200, r.text
    body = r.json()
    assert body["pool_name"] and isinstance(body["instances"], list)


# every REST route of the reference server (its ``server/routers/*.py``, prefix + path), so a
# client of the reference finds each one here
REFERENCE_ROUTES = [
    '/api/backends/config_values',
    '/api/backends/list_types',
    '/api/fleets/list',
    '/api/instances/list',
    '/api/pools/list_instances',
    '/api/project/{project_name}/backends/create',
    '/api/project/{project_name}/backends/create_yaml',
    '/api/project/{project_name}/backends/delete',
    '/api/project/{project_name}/backends/update',
    '/api/project/{project_name}/backends/update_yaml',
    '/api/project/{project_name}/backends/{backend_name}/config_info',
    '/api/project/{project_name}/backends/{backend_name}/get_yaml',
    '/api/project/{project_name}/fleets/create',
    '/api/project/{project_name}/fleets/delete',
    '/api/project/{project_name}/fleets/delete_instances',
    '/api/project/{project_name}/fleets/get',
    '/api/project/{project_name}/fleets/get_plan',
    '/api/project/{project_name}/fleets/list',
    '/api/project/{project_name}/gateways/create',
    '/api/project/{project_name}/gateways/delete',
    '/api/project/{project_name}/gateways/get',
    '/api/project/{project_name}/gateways/list',
    '/api/project/{project_name}/gateways/set_default',
    '/api/project/{project_name}/gateways/set_wildcard_domain',
    '/api/project/{project_name}/logs/poll',
    '/api/project/{project_name}/metrics/job/{run_name}',
    '/api/project/{project_name}/pool/add_remote',
    '/api/project/{project_name}/pool/create',
    '/api/project/{project_name}/pool/delete',
    '/api/project/{project_name}/pool/list',
    '/api/project/{project_name}/pool/remove',
    '/api/project/{project_name}/pool/set_default',
    '/api/project/{project_name}/pool/show',
    '/api/project/{project_name}/repos/delete',
    '/api/project/{project_name}/repos/get',
    '/api/project/{project_name}/repos/init',
    '/api/project/{project_name}/repos/list',
    '/api/project/{project_name}/repos/upload_code',
    '/api/project/{project_name}/runs/apply',
    '/api/project/{project_name}/runs/create_instance',
    '/api/project/{project_name}/runs/delete',
    '/api/project/{project_name}/runs/get',
    '/api/project/{project_name}/runs/get_offers',
    '/api/project/{project_name}/runs/get_plan',
    '/api/project/{project_name}/runs/stop',
    '/api/project/{project_name}/runs/submit',
    '/api/project/{project_name}/secrets/add',
    '/api/project/{project_name}/secrets/delete',
    '/api/project/{project_name}/secrets/get',
    '/api/project/{project_name}/secrets/list',
    '/api/project/{project_name}/volumes/create',
    '/api/project/{project_name}/volumes/delete',
    '/api/project/{project_name}/volumes/get',
    '/api/project/{project_name}/volumes/list',
    '/api/projects/create',
    '/api/projects/delete',
    '/api/projects/list',
    '/api/projects/{project_name}/get',
    '/api/projects/{project_name}/set_members',
    '/api/runs/list',
    '/api/server/get_info',
    '/api/users/create',
    '/api/users/delete',
    '/api/users/get_my_user',
    '/api/users/get_user',
    '/api/users/list',
    '/api/users/refresh_token',
    '/api/users/update',
    '/api/volumes/list',
]


def test_openapi_schema_covers_reference_routes(client):
    import re

    r = client.get("/api/openapi.json")
    assert r.status_code == 200, r.text[:500]
    norm = lambda p: re.sub(r"\{[^}]+\}", "{}", p)  # noqa: E731
    ours = {norm(p) for p in r.json()["paths"]}
    missing = [p for p in REFERENCE_ROUTES if norm(p) not in ours]
    assert not missing, missing


# ---- default permissions (server config.yml) ---------------------------------------------------
def test_default_permissions_restrict_projects_and_ssh_fleets(client, tmp_path):
    """``default_permissions`` of the server config: with both switches off a non-admin user can
    neither create projects nor create/delete SSH fleets, a project admin still manages SSH fleets,
    and the derived permissions are reported on users and members."""
    from dstack_amd.server.services import permissions
    from dstack_amd.server.services.config import ServerConfigManager

    cfg = tmp_path / "config.yml"
    cfg.write_text("default_permissions:\n  allow_non_admins_create_projects: false\n"
                   "  allow_non_admins_manage_ssh_fleets: false\n")
    ServerConfigManager(cfg).load_config()
    try:
        u = client.post("/api/users/create", json={"username": "erin"}).json()
        assert u["permissions"] == {"can_create_projects": False}
        erin = {"Authorization": f"Bearer {u['creds']['token']}"}
        r = client.post("/api/projects/create", json={"project_name": "erins"}, headers=erin)
        assert r.status_code == 403, r.text
        assert client.post("/api/users/get_my_user").json()["permissions"]["can_create_projects"]
        r = client.post("/api/projects/main/set_members",
                        json={"members": [{"username": "admin", "project_role": "admin"},
                                          {"username": "erin", "project_role": "user"}]})
        assert r.status_code == 200, r.text
        members = {m["user"]["username"]: m for m in client.post("/api/projects/main/get").json()["members"]}
        assert members["erin"]["permissions"] == {"can_manage_ssh_fleets": False}
        assert members["admin"]["permissions"] == {"can_manage_ssh_fleets": True}
        key = {"public": "ssh-ed25519 AAAA", "private": "-----BEGIN OPENSSH PRIVATE KEY-----\nx\n"
                                                       "-----END OPENSSH PRIVATE KEY-----\n"}
        spec = {"spec": {"configuration": {"type": "fleet", "name": "onprem2",
                                           "ssh_config": {"user": "ubuntu", "ssh_key": key, "hosts": ["10.0.0.9"]}},
                         "profile": {"name": "default"}}}
        assert client.post("/api/project/main/fleets/create", json=spec, headers=erin).status_code == 403
        assert client.post("/api/project/main/fleets/create", json=spec).status_code == 200
        r = client.post("/api/project/main/fleets/delete", json={"names": ["onprem2"]}, headers=erin)
        assert r.status_code == 403
        # the pool API's SSH-host door is closed by the same rule
        host = {"host": "10.0.0.10", "port": 22, "ssh_user": "ubuntu", "ssh_keys": [key], "instance_name": "h10"}
        assert client.post("/api/project/main/pool/add_remote", json=host, headers=erin).status_code == 403
        r = client.post("/api/project/main/pool/add_remote", json=host)
        assert r.status_code == 200, r.text
        pool = client.post("/api/project/main/pool/list").json()[0]["name"]
        r = client.post("/api/project/main/pool/remove", json={"pool_name": pool, "instance_name": r.json()["name"],
                                                               "force": True}, headers=erin)
        assert r.status_code == 403, r.text
        # promoted to project admin: allowed
        client.post("/api/projects/main/set_members",
                    json={"members": [{"username": "admin", "project_role": "admin"},
                                      {"username": "erin", "project_role": "admin"}]})
        r = client.post("/api/project/main/fleets/delete", json={"names": ["onprem2"]}, headers=erin)
        assert r.status_code == 200, r.text
    finally:
        permissions.set_default_permissions(None)
    assert client.post("/api/projects/create", json={"project_name": "erins"}, headers=erin).status_code == 200
