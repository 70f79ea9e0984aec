"""Runs router, case by case against the reference's ``routers/test_runs.py`` (mapping:
``docs/reference/test-parity.md``): get by name / deleted run by id, plans that honour
``privileged`` and instance mounts, apply create-vs-update, submit without a name / with a bad name /
an unknown repo, stop in each state, delete rules, ``create_instance``, and where a service's URL
points (in-server proxy or a gateway)."""

from __future__ import annotations

import pytest

from dstack_amd.server.db import session_scope
from dstack_amd.server.models import RunModel
from tests.test_backends_api import VALID


def _repo(client, repo="virt"):
    r = client.post("/api/project/main/repos/init", json={"repo_id": repo, "repo_info": {"repo_type": "virtual"}})
    assert r.status_code == 200, r.text


def _spec(name, conf=None, repo="virt"):
    conf = conf or {"type": "task", "commands": ["echo hi"]}
    spec = {"repo_id": repo, "repo_data": {"repo_type": "virtual"}, "configuration": conf, "ssh_key_pub": ""}
    if name is not None:
        spec["run_name"] = name
    return {"run_spec": spec}


def _submit(client, name, conf=None):
    r = client.post("/api/project/main/runs/submit", json=_spec(name, conf))
    assert r.status_code == 200, r.text
    return r.json()


def _backends(client, *types):
    for t in types:
        assert client.post("/api/project/main/backends/create", json=VALID[t]).status_code == 200


def _offer_backends(plan):
    return {o["backend"] for o in plan["job_plans"][0]["offers"]}


def _set_status(name, status):
    with session_scope() as s:
        s.query(RunModel).filter_by(run_name=name).one().status = status


# ---- get ----------------------------------------------------------------------------------------
def test_get_run_by_name(client):
    _repo(client)
    _submit(client, "named")
    got = client.post("/api/project/main/runs/get", json={"run_name": "named"})
    assert got.status_code == 200
    run = got.json()
    assert run["run_spec"]["run_name"] == "named" and run["status"] == "submitted"
    assert run["user"] == "admin" and run["project_name"] == "main"
    assert len(run["jobs"]) == 1 and run["jobs"][0]["job_submissions"][0]["submission_num"] == 0


def test_get_deleted_run_by_id_but_not_by_name(client):
    _repo(client)
    run = _submit(client, "to-delete")
    client.post("/api/project/main/runs/stop", json={"runs_names": ["to-delete"], "abort": True})
    _set_status("to-delete", "terminated")
    assert client.post("/api/project/main/runs/delete", json={"runs_names": ["to-delete"]}).status_code == 200
    assert client.post("/api/project/main/runs/get", json={"run_name": "to-delete"}).status_code == 400
    got = client.post("/api/project/main/runs/get", json={"id": run["id"]})
    assert got.status_code == 200 and got.json()["run_spec"]["run_name"] == "to-delete"


# ---- plan ---------------------------------------------------------------------------------------
def test_plan_privileged_false_offers_every_backend(client):
    _repo(client)
    _backends(client, "aws", "runpod")
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("p0", {"type": "task", "commands": ["x"],
                                                                           "resources": {"gpu": "MI300X"}}))
    assert plan.status_code == 200, plan.text
    assert "runpod" in _offer_backends(plan.json())


def test_plan_privileged_true_drops_container_backends(client):
    """Container clouds cannot run a privileged container (reference: offers only from backends
    that can create instances)."""
    _repo(client)
    _backends(client, "aws", "runpod")
    conf = {"type": "task", "commands": ["x"], "privileged": True}
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("p1", conf)).json()
    backends = _offer_backends(plan)
    assert backends and "runpod" not in backends and "vastai" not in backends


def test_plan_instance_volumes_need_vm_backends(client):
    _repo(client)
    _backends(client, "aws", "runpod")
    conf = {"type": "task", "commands": ["x"], "volumes": [{"instance_path": "/mnt/data", "path": "/data"}]}
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("p2", conf)).json()
    backends = _offer_backends(plan)
    assert backends and "runpod" not in backends


def test_plan_update_action_for_updatable_fields(client):
    _repo(client)
    svc = {"type": "service", "commands": ["serve"], "port": 8000, "replicas": 1}
    _submit(client, "svc", svc)
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("svc", dict(svc, replicas=2))).json()
    assert plan["action"] == "update" and plan["current_resource"]["run_spec"]["run_name"] == "svc"


def test_plan_create_action_for_non_updatable_fields(client):
    _repo(client)
    svc = {"type": "service", "commands": ["serve"], "port": 8000}
    _submit(client, "svc2", svc)
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("svc2", dict(svc, commands=["serve2"]))).json()
    assert plan["action"] == "create"


# ---- apply --------------------------------------------------------------------------------------
def test_apply_submits_new_run_without_current_resource(client):
    _repo(client)
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("fresh")).json()
    r = client.post("/api/project/main/runs/apply", json={"plan": {"run_spec": plan["run_spec"],
                                                                   "current_resource": None}, "force": False})
    assert r.status_code == 200, r.text
    assert r.json()["run_spec"]["run_name"] == "fresh" and r.json()["status"] == "submitted"


def test_apply_updates_run_in_place(client):
    _repo(client)
    svc = {"type": "service", "commands": ["serve"], "port": 8000, "replicas": 1}
    first = _submit(client, "upd", svc)
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("upd", dict(svc, replicas=3))).json()
    r = client.post("/api/project/main/runs/apply", json={"plan": {"run_spec": plan["run_spec"],
                                                                   "current_resource": plan["current_resource"]},
                                                          "force": False})
    assert r.status_code == 200, r.text
    assert r.json()["id"] == first["id"]  # same run, updated
    assert r.json()["run_spec"]["configuration"]["replicas"]["min"] == 3


# ---- submit -------------------------------------------------------------------------------------
def test_submit_run(client):
    _repo(client)
    run = _submit(client, "sub1")
    assert run["status"] == "submitted" and run["run_spec"]["run_name"] == "sub1"
    assert run["jobs"][0]["job_spec"]["job_name"].startswith("sub1-0")


def test_submit_run_without_name_generates_one(client):
    _repo(client)
    r = client.post("/api/project/main/runs/submit", json=_spec(None))
    assert r.status_code == 200, r.text
    name = r.json()["run_spec"]["run_name"]
    assert name and "-" in name


@pytest.mark.parametrize("bad", ["Bad_Name", "x" * 100, "-lead", "sp ace"])
def test_submit_run_bad_name_400(client, bad):
    _repo(client)
    assert client.post("/api/project/main/runs/submit", json=_spec(bad)).status_code == 400


def test_submit_run_unknown_repo_400(client):
    """A local/remote repo must be initialised first (a virtual repo has nothing to upload)."""
    body = _spec("norepo", repo="does-not-exist")
    body["run_spec"]["repo_data"] = {"repo_type": "local", "repo_dir": "/tmp/x"}
    r = client.post("/api/project/main/runs/submit", json=body)
    assert r.status_code == 400 and "Repo does-not-exist does not exist" in r.text


# ---- stop ---------------------------------------------------------------------------------------
def test_stop_submitted_run_terminates(client):
    _repo(client)
    _submit(client, "stop-sub")
    assert client.post("/api/project/main/runs/stop", json={"runs_names": ["stop-sub"], "abort": False}
                       ).status_code == 200
    run = client.post("/api/project/main/runs/get", json={"run_name": "stop-sub"}).json()
    assert run["status"] in ("terminating", "terminated")
    assert run["termination_reason"] == "stopped_by_user"


def test_stop_running_run_terminates(client):
    _repo(client)
    _submit(client, "stop-run")
    _set_status("stop-run", "running")
    client.post("/api/project/main/runs/stop", json={"runs_names": ["stop-run"], "abort": True})
    run = client.post("/api/project/main/runs/get", json={"run_name": "stop-run"}).json()
    assert run["status"] == "terminating" and run["termination_reason"] == "aborted_by_user"


def test_stop_leaves_finished_runs_unchanged(client):
    _repo(client)
    _submit(client, "stop-done")
    _set_status("stop-done", "done")
    assert client.post("/api/project/main/runs/stop", json={"runs_names": ["stop-done"], "abort": True}
                       ).status_code == 200
    run = client.post("/api/project/main/runs/get", json={"run_name": "stop-done"}).json()
    assert run["status"] == "done" and run["termination_reason"] is None


# ---- delete -------------------------------------------------------------------------------------
def test_delete_runs(client):
    _repo(client)
    _submit(client, "del1")
    _set_status("del1", "failed")
    assert client.post("/api/project/main/runs/delete", json={"runs_names": ["del1"]}).status_code == 200
    assert client.post("/api/runs/list", json={}).json() == []


def test_delete_active_run_400(client):
    _repo(client)
    _submit(client, "del2")
    r = client.post("/api/project/main/runs/delete", json={"runs_names": ["del2"]})
    assert r.status_code == 400
    assert len(client.post("/api/runs/list", json={}).json()) == 1


# ---- create_instance ----------------------------------------------------------------------------
def test_create_instance(client):
    _backends(client, "aws")
    r = client.post("/api/project/main/runs/create_instance", json={
        "profile": {"name": "default", "backends": ["aws"]},
        "requirements": {"resources": {"gpu": "H100:8"}}})
    assert r.status_code == 200, r.text
    inst = r.json()
    assert inst["backend"] == "aws" and inst["status"] in ("pending", "provisioning")
    listed = client.post("/api/instances/list", json={}).json()
    assert [i["name"] for i in listed] == [inst["name"]]


def test_create_instance_without_capable_backends_400(client):
    """Only container / local backends configured: nothing can create a bare instance."""
    _backends(client, "runpod")
    r = client.post("/api/project/main/runs/create_instance", json={
        "profile": {"name": "default", "backends": ["runpod"]}, "requirements": {"resources": {}}})
    assert r.status_code == 400
    assert "create" in r.text.lower() or "offer" in r.text.lower() or "backend" in r.text.lower()


# ---- services -----------------------------------------------------------------------------------
def _service(**kw):
    return {"type": "service", "commands": ["serve"], "port": 8000, **kw}


def test_service_url_in_server_proxy_without_gateway(client):
    _repo(client)
    run = _submit(client, "svc-proxy", _service())
    assert run["service"]["url"] == "/proxy/services/main/svc-proxy/"


def _gateways(client, *named):
    """Running gateways (name, is_default) with ``<name>.example`` wildcard domains."""
    from dstack_amd.server.models import BackendModel, GatewayModel, ProjectModel

    _backends(client, "aws")
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="main").one()
        backend = s.query(BackendModel).filter_by(type="aws").one()
        for name, default in named:
            gw = GatewayModel(name=name, region="us-east-1", wildcard_domain=f"{name}.example", status="running",
                              project_id=project.id, backend_id=backend.id)
            s.add(gw)
            s.flush()
            if default:
                project.default_gateway_id = gw.id


@pytest.mark.parametrize("gateways,specified,url,model_url", [
    ([("default-gw", True), ("other-gw", False)], None, "https://svc.default-gw.example",
     "https://gateway.default-gw.example"),
    ([("default-gw", True), ("other-gw", False)], "other-gw", "https://svc.other-gw.example",
     "https://gateway.other-gw.example"),
    ([("other-gw", False)], None, "/proxy/services/main/svc/", "/proxy/models/main/"),
    ([("default-gw", True)], False, "/proxy/services/main/svc/", "/proxy/models/main/"),
], ids=["default-gateway", "specified-gateway", "in-server-no-default", "in-server-specified"])
def test_service_submitted_to_the_right_proxy(client, monkeypatch, gateways, specified, url, model_url):
    from dstack_amd.server.services import gateways as gateways_services

    registered = []
    monkeypatch.setattr(gateways_services, "gateway_register_service", lambda s, run: registered.append(run.run_name))
    _repo(client)
    _gateways(client, *gateways)
    conf = _service(model={"type": "chat", "name": "m", "format": "openai"})
    if specified is not None:
        conf["gateway"] = specified
    run = _submit(client, "svc", conf)
    assert run["service"]["url"] == url
    assert run["service"]["model"]["base_url"] == model_url
    assert registered == (["svc"] if url.startswith("https://") else [])


def test_service_with_unknown_gateway_400(client):
    _repo(client)
    r = client.post("/api/project/main/runs/submit", json=_spec("svc-bad", _service(gateway="nosuchgw")))
    assert r.status_code == 400 and "Gateway nosuchgw does not exist" in r.text


def test_service_gateway_true_is_a_validation_error(client):
    """``gateway: true`` is not a gateway name: rejected by the configuration schema (422)."""
    _repo(client)
    r = client.post("/api/project/main/runs/submit", json=_spec("svc-true", _service(gateway=True)))
    assert r.status_code == 422
