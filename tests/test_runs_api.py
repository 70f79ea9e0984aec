"""Runs REST API beyond the basics (reference: ``src/tests/_internal/server/routers/test_runs.py``):
listing filters and keyset pagination, get by id, plans for every run type, apply-update in place
of a service's replicas/scaling, delete rules, permissions of non-members, env/secret handling in
job specs."""

from __future__ import annotations

import uuid
from datetime import timedelta

import pytest

from dstack_amd.server.db import session_scope
from dstack_amd.server.models import RunModel
from tests.conftest import ADMIN_TOKEN


def _spec(name, conf=None, repo="virt"):
    conf = conf or {"type": "task", "commands": ["echo hi"]}
    return {"run_spec": {"run_name": name, "repo_id": repo, "repo_data": {"repo_type": "virtual"},
                         "configuration": conf, "ssh_key_pub": ""}}


def _repo(client, repo="virt", project="main", headers=None):
    r = client.post(f"/api/project/{project}/repos/init", json={"repo_id": repo, "repo_info": {"repo_type": "virtual"}},
                    headers=headers)
    assert r.status_code == 200, r.text


def _submit(client, name, conf=None, project="main", headers=None, repo="virt"):
    r = client.post(f"/api/project/{project}/runs/submit", json=_spec(name, conf, repo), headers=headers)
    assert r.status_code == 200, r.text
    return r.json()


def _user(client, name, role="user"):
    u = client.post("/api/users/create", json={"username": name, "global_role": role}).json()
    return {"Authorization": f"Bearer {u['creds']['token']}"}


def _names(runs):
    return [r["run_spec"]["run_name"] for r in runs]


# ---- listing ------------------------------------------------------------------------------------
def test_list_runs_newest_first_and_keyset_pages(client):
    _repo(client)
    for i in range(5):
        _submit(client, f"run-{i}")
    # force equal submitted_at for two runs to exercise the (submitted_at, id) tie-break
    with session_scope() as s:
        runs = {r.run_name: r for r in s.query(RunModel)}
        runs["run-3"].submitted_at = runs["run-2"].submitted_at
    all_runs = client.post("/api/runs/list", json={}).json()
    assert len(all_runs) == 5
    subs = [(r["submitted_at"], r["id"]) for r in all_runs]
    assert subs == sorted(subs, reverse=True)
    page, seen = None, []
    while True:
        body = {"limit": 2}
        if page:
            body.update(prev_submitted_at=page[-1]["submitted_at"], prev_run_id=page[-1]["id"])
        page = client.post("/api/runs/list", json=body).json()
        if not page:
            break
        assert len(page) <= 2
        seen += _names(page)
    assert seen == _names(all_runs)  # no duplicates, nothing skipped across the tie
    asc = client.post("/api/runs/list", json={"ascending": True}).json()
    assert _names(asc) == list(reversed(_names(all_runs)))


def test_list_runs_filters(client):
    _repo(client)
    _repo(client, "other")
    bob = _user(client, "bob")
    client.post("/api/projects/main/set_members", json={"members": [
        {"username": "admin", "project_role": "admin"}, {"username": "bob", "project_role": "user"}]})
    _submit(client, "by-admin")
    _submit(client, "by-bob", headers=bob)
    _submit(client, "other-repo", repo="other")
    client.post("/api/project/main/runs/stop", json={"runs_names": ["other-repo"], "abort": True})
    with session_scope() as s:
        r = s.query(RunModel).filter_by(run_name="other-repo").one()
        r.status = "terminated"
    assert set(_names(client.post("/api/runs/list", json={"username": "bob"}).json())) == {"by-bob"}
    assert set(_names(client.post("/api/runs/list", json={"project_name": "main", "repo_id": "other"}).json())) == {
        "other-repo"}
    assert client.post("/api/runs/list", json={"repo_id": "other"}).json() == []  # repo needs a project
    active = set(_names(client.post("/api/runs/list", json={"only_active": True}).json()))
    assert active == {"by-admin", "by-bob"}
    assert client.post("/api/runs/list", json={"username": "nobody"}).status_code == 400
    r = client.post("/api/runs/list", json={"project_name": "main", "repo_id": "missing"})
    assert r.status_code == 400


def test_non_member_sees_no_runs_and_cannot_read_them(client):
    _repo(client)
    _submit(client, "secret-run")
    eve = _user(client, "eve")
    assert client.post("/api/runs/list", json={}, headers=eve).json() == []
    assert client.post("/api/project/main/runs/get", json={"run_name": "secret-run"}, headers=eve).status_code == 403
    assert client.post("/api/project/main/runs/submit", json=_spec("x"), headers=eve).status_code == 403


# ---- get / plan / apply -----------------------------------------------------------------------
def test_get_run_by_id_and_unknown(client):
    _repo(client)
    run = _submit(client, "by-id")
    got = client.post("/api/project/main/runs/get", json={"id": run["id"]}).json()
    assert got["run_spec"]["run_name"] == "by-id"
    r = client.post("/api/project/main/runs/get", json={"id": str(uuid.uuid4())})
    assert r.status_code == 400
    assert client.post("/api/project/main/runs/get", json={"run_name": "nope"}).status_code == 400


@pytest.mark.parametrize("conf,expect_jobs", [
    ({"type": "task", "commands": ["x"], "nodes": 3}, 3),
    ({"type": "service", "commands": ["x"], "port": 8000, "replicas": "1..3",
      "scaling": {"metric": "rps", "target": 10}}, 1),
    ({"type": "dev-environment", "ide": "vscode"}, 1),
])
def test_plan_for_each_run_type(client, conf, expect_jobs):
    _repo(client)
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("planned", conf))
    assert plan.status_code == 200, plan.text
    body = plan.json()
    assert body["action"] == "create" and body["current_resource"] is None
    assert len(body["job_plans"]) == expect_jobs
    spec = body["job_plans"][0]["job_spec"]
    assert spec["image_name"]  # a ROCm base image when none is given
    if conf["type"] == "dev-environment":
        assert spec["max_duration"] is not None


def test_plan_of_active_run_is_update(client):
    _repo(client)
    _submit(client, "svc", {"type": "service", "commands": ["x"], "port": 8000, "replicas": 1})
    body = client.post("/api/project/main/runs/get_plan", json=_spec(
        "svc", {"type": "service", "commands": ["x"], "port": 8000, "replicas": 2})).json()
    assert body["action"] == "update" and body["current_resource"]["run_spec"]["run_name"] == "svc"


def test_apply_updates_service_replicas_in_place(client):
    _repo(client)
    first = _submit(client, "svc", {"type": "service", "commands": ["x"], "port": 8000, "replicas": 1})
    plan = client.post("/api/project/main/runs/get_plan", json=_spec(
        "svc", {"type": "service", "commands": ["x"], "port": 8000, "replicas": "2..4",
                "scaling": {"metric": "rps", "target": 5}})).json()
    r = client.post("/api/project/main/runs/apply", json={"plan": {"run_spec": plan["run_spec"],
                                                                  "current_resource": plan["current_resource"]}})
    assert r.status_code == 200, r.text
    assert r.json()["id"] == first["id"]  # same run, updated
    with session_scope() as s:
        run = s.query(RunModel).filter_by(run_name="svc", deleted=False).one()
        assert run.desired_replica_count == 2  # clamped into the new 2..4 range


def test_apply_with_changed_commands_stops_old_run(client):
    _repo(client)
    _submit(client, "tt", {"type": "task", "commands": ["a"]})
    plan = client.post("/api/project/main/runs/get_plan", json=_spec("tt", {"type": "task", "commands": ["b"]})).json()
    assert plan["action"] == "create" and plan["current_resource"] is not None  # not updatable in place
    r = client.post("/api/project/main/runs/apply", json={"plan": {"run_spec": plan["run_spec"],
                                                                  "current_resource": plan["current_resource"]}})
    assert r.status_code == 400 and "Stop the run first" in r.text
    assert client.post("/api/project/main/runs/get", json={"run_name": "tt"}).json()["status"] == "submitted"
    # the client stops it; once finished, applying the new spec creates a new run
    client.post("/api/project/main/runs/stop", json={"runs_names": ["tt"], "abort": True})
    with session_scope() as s:
        s.query(RunModel).filter_by(run_name="tt", deleted=False).one().status = "terminated"
    r = client.post("/api/project/main/runs/apply", json={"plan": {"run_spec": plan["run_spec"]}})
    assert r.status_code == 200, r.text
    assert r.json()["jobs"][0]["job_spec"]["commands"][-1].endswith("b")


def test_in_place_update_rules(client):
    """Reference ``_check_can_update_run_spec``: only services, and only replicas / scaling /
    strip_prefix (plus new code); an identical active task is not "updated"."""
    _repo(client)
    _submit(client, "svc2", {"type": "service", "commands": ["x"], "port": 8000})
    plan = lambda name, conf: client.post("/api/project/main/runs/get_plan", json=_spec(name, conf)).json()  # noqa: E731
    assert plan("svc2", {"type": "service", "commands": ["x"], "port": 8000, "strip_prefix": False})["action"] == "update"
    assert plan("svc2", {"type": "service", "commands": ["x"], "port": 8001})["action"] == "create"
    assert plan("svc2", {"type": "service", "commands": ["x"], "port": 8000, "env": {"A": "1"}})["action"] == "create"
    _submit(client, "tsk", {"type": "task", "commands": ["a"]})
    assert plan("tsk", {"type": "task", "commands": ["a"]})["action"] == "create"


def test_apply_stale_plan_rejected_unless_forced(client):
    _repo(client)
    _submit(client, "svc", {"type": "service", "commands": ["x"], "port": 8000})
    plan = client.post("/api/project/main/runs/get_plan", json=_spec(
        "svc", {"type": "service", "commands": ["x"], "port": 8000, "replicas": 2})).json()
    stale = dict(plan["current_resource"], id=str(uuid.uuid4()))
    body = {"plan": {"run_spec": plan["run_spec"], "current_resource": stale}}
    assert client.post("/api/project/main/runs/apply", json=body).status_code == 400
    assert client.post("/api/project/main/runs/apply", json=dict(body, force=True)).status_code == 200


def test_resubmitting_finished_run_name_replaces_it(client):
    _repo(client)
    old = _submit(client, "again")
    with session_scope() as s:
        s.query(RunModel).filter_by(run_name="again").one().status = "done"
    new = _submit(client, "again")
    assert new["id"] != old["id"]
    assert _names(client.post("/api/runs/list", json={}).json()) == ["again"]


# ---- stop / delete ------------------------------------------------------------------------------
def test_delete_finished_runs_only(client):
    _repo(client)
    _submit(client, "keep")
    _submit(client, "gone")
    with session_scope() as s:
        s.query(RunModel).filter_by(run_name="gone").one().status = "failed"
    assert client.post("/api/project/main/runs/delete", json={"runs_names": ["keep"]}).status_code == 400
    assert client.post("/api/project/main/runs/delete", json={"runs_names": ["gone"]}).status_code == 200
    assert _names(client.post("/api/runs/list", json={}).json()) == ["keep"]
    # stopping unknown or finished runs is a no-op
    assert client.post("/api/project/main/runs/stop", json={"runs_names": ["nope"]}).status_code == 200


def test_invalid_run_name_rejected(client):
    _repo(client)
    r = client.post("/api/project/main/runs/submit", json=_spec("Bad_Name"))
    assert r.status_code == 400


# ---- job specs: env, secrets, interpolation -------------------------------------------------------
def test_job_spec_env_and_secret_interpolation(client):
    _repo(client)
    client.post("/api/project/main/secrets/add", json={"name": "HF_TOKEN", "value": "hf-123"})
    conf = {"type": "task", "commands": ["echo $MODEL"], "env": {"MODEL": "llama", "TOKEN": "${{ secrets.HF_TOKEN }}"},
            "resources": {"gpu": "MI355X:8", "shm_size": "64GB"}}
    run = _submit(client, "envs", conf)
    spec = run["jobs"][0]["job_spec"]
    assert spec["env"]["MODEL"] == "llama"
    assert spec["env"]["TOKEN"] == "hf-123"
    gpu = spec["requirements"]["resources"]["gpu"]
    assert gpu["count"]["min"] == 8 and "MI355X" in gpu["name"]


def test_run_submitted_at_and_timings_exposed(client):
    _repo(client)
    run = _submit(client, "timed")
    sub = run["jobs"][0]["job_submissions"][0]
    assert sub["submitted_at"] and sub["status"] == "submitted"
    assert run["submitted_at"]


def test_admin_token_header_required_everywhere(client):
    r = client.post("/api/runs/list", json={}, headers={"Authorization": f"Bearer {ADMIN_TOKEN}x"})
    assert r.status_code in (401, 403)


def test_prev_submitted_at_without_id_is_strict(client):
    _repo(client)
    a = _submit(client, "a1")
    _submit(client, "a2")
    with session_scope() as s:
        r = s.query(RunModel).filter_by(run_name="a2").one()
        r.submitted_at = r.submitted_at + timedelta(seconds=5)
    newest = client.post("/api/runs/list", json={"limit": 1}).json()
    assert _names(newest) == ["a2"]
    rest = client.post("/api/runs/list", json={"prev_submitted_at": newest[0]["submitted_at"]}).json()
    assert _names(rest) == ["a1"] and rest[0]["id"] == a["id"]
