"""Fleets, gateways, volumes, instances, pools, logs, metrics and repos routers, case by case
against the reference's ``routers/test_{fleets,gateways,volumes,instances,pools,logs,metrics,repos}.py``
(mapping: ``docs/reference/test-parity.md``).  Unauthenticated / non-member / non-admin cases are in
``test_api_access_matrix.py``."""

from __future__ import annotations

import base64
import json
import uuid

from dstack_amd.core.models.instances import InstanceStatus
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import FleetModel, GatewayModel, InstanceModel, ProjectModel
from tests.test_backends_api import VALID
from tests.test_fleets_volumes_api import _create, _fleet, _ssh


def _backend(client, t="aws"):
    types = {b["name"] for b in client.post("/api/projects/main/get").json()["backends"]}
    if t not in types:
        assert client.post("/api/project/main/backends/create", json=VALID[t]).status_code == 200


def _user(client, name, role="user", project_role=None):
    u = client.post("/api/users/create", json={"username": name, "global_role": role}).json()
    h = {"Authorization": f"Bearer {u['creds']['token']}"}
    if project_role:
        members = [{"username": m["user"]["username"], "project_role": m["project_role"]}
                   for m in client.post("/api/projects/main/get").json()["members"]]
        client.post("/api/projects/main/set_members",
                    json={"members": members + [{"username": name, "project_role": project_role}]})
    return h


# ---- fleets -------------------------------------------------------------------------------------
def test_list_project_fleets(client):
    _create(client, _ssh(name="f1", hosts=["10.0.2.1"]))
    _create(client, _ssh(name="f2", hosts=["10.0.2.2"]))
    fleets = client.post("/api/project/main/fleets/list").json()
    assert sorted(f["name"] for f in fleets) == ["f1", "f2"]
    assert all(f["project_name"] == "main" and f["spec"]["configuration"]["ssh_config"] for f in fleets)


def test_get_fleet_by_id_and_by_name(client):
    f = _create(client, _ssh(name="byid", hosts=["10.0.2.3"]))
    by_id = client.post("/api/project/main/fleets/get", json={"id": f["id"]})
    assert by_id.status_code == 200 and by_id.json()["name"] == "byid"
    by_name = client.post("/api/project/main/fleets/get", json={"name": "byid"})
    assert by_name.status_code == 200 and by_name.json()["id"] == f["id"]


def test_deleted_fleet_not_returned_by_name_but_by_id(client):
    f = _create(client, _ssh(name="gonefleet", hosts=["10.0.2.4"]))
    with session_scope() as s:
        row = s.get(FleetModel, uuid.UUID(f["id"]))
        row.deleted = True
    assert client.post("/api/project/main/fleets/get", json={"name": "gonefleet"}).status_code == 400
    assert client.post("/api/project/main/fleets/get", json={"id": f["id"]}).json()["name"] == "gonefleet"
    assert client.post("/api/project/main/fleets/get", json={"name": "never-existed"}).status_code == 400


def test_create_cloud_fleet(client):
    _backend(client)
    r = client.post("/api/project/main/fleets/create", json=_fleet({"name": "cloud", "nodes": 2,
                                                                     "resources": {"gpu": "H100:8"}}))
    assert r.status_code == 200, r.text
    f = r.json()
    assert f["status"] == "active" and len(f["instances"]) == 2
    assert {i["status"] for i in f["instances"]} == {"pending"}
    assert [i["instance_num"] for i in f["instances"]] == [0, 1]


def test_create_ssh_fleet(client):
    f = _create(client, _ssh(name="sshf", hosts=["10.0.3.1", {"hostname": "10.0.3.2", "port": 2222}]))
    assert f["spec"]["configuration"]["ssh_config"]["hosts"][1]["port"] == 2222
    insts = f["instances"]
    assert [i["instance_num"] for i in insts] == [0, 1] and all(i["backend"] == "remote" for i in insts)
    assert all(i["status"] == "pending" for i in insts)


def test_create_ssh_fleet_with_bad_key_400(client):
    body = _ssh(name="badkey")
    body["spec"]["configuration"]["ssh_config"]["ssh_key"] = {"public": "", "private": "123"}
    r = client.post("/api/project/main/fleets/create", json=body)
    assert r.status_code == 400


def test_delete_fleets_terminates_their_instances(client):
    _create(client, _ssh(name="todel", hosts=["10.0.4.1", "10.0.4.2"]))
    assert client.post("/api/project/main/fleets/delete", json={"names": ["todel"]}).status_code == 200
    with session_scope() as s:
        f = s.query(FleetModel).filter_by(name="todel").one()
        assert f.status == "terminating"
        assert {i.status for i in f.instances} == {InstanceStatus.TERMINATING.value}


def test_delete_fleet_instances(client):
    _create(client, _ssh(name="partial", hosts=["10.0.5.1", "10.0.5.2"]))
    r = client.post("/api/project/main/fleets/delete_instances", json={"name": "partial", "instance_nums": [1]})
    assert r.status_code == 200, r.text
    with session_scope() as s:
        f = s.query(FleetModel).filter_by(name="partial").one()
        by_num = {i.instance_num: i.status for i in f.instances}
        assert by_num == {0: InstanceStatus.PENDING.value, 1: InstanceStatus.TERMINATING.value}
        assert f.status != "terminating"


def test_delete_busy_fleet_instances_400(client):
    _create(client, _ssh(name="busyf", hosts=["10.0.6.1", "10.0.6.2"]))
    with session_scope() as s:
        inst = s.query(InstanceModel).filter_by(instance_num=1).one()
        inst.status = InstanceStatus.BUSY.value
        inst.busy_blocks = 1
    r = client.post("/api/project/main/fleets/delete_instances", json={"name": "busyf", "instance_nums": [1]})
    assert r.status_code == 400
    with session_scope() as s:
        f = s.query(FleetModel).filter_by(name="busyf").one()
        assert all(i.status != InstanceStatus.TERMINATING.value for i in f.instances)
        assert f.status != "terminating"


def test_ssh_fleet_instance_deletes_need_permission(client):
    from dstack_amd.server.services import permissions

    _create(client, _ssh(name="perm", hosts=["10.0.7.1", "10.0.7.2"]))
    h = _user(client, "noperm", project_role="user")
    permissions.set_default_permissions({"allow_non_admins_manage_ssh_fleets": False})
    try:
        r = client.post("/api/project/main/fleets/delete_instances", json={"name": "perm", "instance_nums": [0]},
                        headers=h)
        assert r.status_code == 403
        # deleting the whole SSH fleet needs the same permission
        assert client.post("/api/project/main/fleets/delete", json={"names": ["perm"]}, headers=h).status_code == 403
        assert client.post("/api/project/main/fleets/get", json={"name": "perm"}).json()["status"] != "terminating"
    finally:
        permissions.set_default_permissions(None)


def test_fleet_plan(client):
    _backend(client)
    spec = _fleet({"name": "planned", "nodes": 1, "resources": {"gpu": "H100:8"}})["spec"]
    r = client.post("/api/project/main/fleets/get_plan", json={"spec": spec})
    assert r.status_code == 200, r.text
    plan = r.json()
    assert plan["spec"]["configuration"]["name"] == "planned" and plan["current_resource"] is None
    assert plan["offers"] and all(o["backend"] == "aws" for o in plan["offers"])
    assert plan["total_offers"] >= len(plan["offers"])


# ---- gateways -----------------------------------------------------------------------------------
def _gw(client, name="gw", default=False, domain="example.com"):
    _backend(client)
    with session_scope() as s:
        from dstack_amd.server.models import BackendModel

        project = s.query(ProjectModel).filter_by(name="main").one()
        backend = s.query(BackendModel).filter_by(type="aws").one()
        g = GatewayModel(name=name, region="us-east-1", wildcard_domain=domain, status="running",
                         project_id=project.id, backend_id=backend.id,
                         configuration=json.dumps({"type": "gateway", "name": name, "backend": "aws",
                                                   "region": "us-east-1", "domain": domain}))
        s.add(g)
        s.flush()
        if default:
            project.default_gateway_id = g.id


def test_list_and_get_gateways(client):
    _gw(client, "gw-a", default=True)
    lst = client.post("/api/project/main/gateways/list").json()
    assert [g["name"] for g in lst] == ["gw-a"]
    g = lst[0]
    assert g["backend"] == "aws" and g["region"] == "us-east-1" and g["wildcard_domain"] == "example.com"
    assert g["default"] is True
    got = client.post("/api/project/main/gateways/get", json={"name": "gw-a"})
    assert got.status_code == 200 and got.json()["name"] == "gw-a"


def test_get_missing_gateway_400(client):
    assert client.post("/api/project/main/gateways/get", json={"name": "nope"}).status_code == 400


def test_create_gateway(client, monkeypatch):
    _backend(client)
    r = client.post("/api/project/main/gateways/create", json={"configuration": {
        "type": "gateway", "name": "new-gw", "backend": "aws", "region": "us-east-1", "domain": "apps.example.com"}})
    assert r.status_code == 200, r.text
    g = r.json()
    assert g["name"] == "new-gw" and g["status"] == "submitted" and g["wildcard_domain"] == "apps.example.com"
    # the first gateway of a project becomes its default
    assert g["default"] is True


def test_create_gateway_without_name_generates_one(client):
    _backend(client)
    r = client.post("/api/project/main/gateways/create", json={"configuration": {
        "type": "gateway", "backend": "aws", "region": "us-east-1", "domain": "x.example.com"}})
    assert r.status_code == 200, r.text
    assert r.json()["name"]


def test_create_gateway_on_unconfigured_backend_400(client):
    r = client.post("/api/project/main/gateways/create", json={"configuration": {
        "type": "gateway", "name": "g", "backend": "gcp", "region": "us-central1", "domain": "e.com"}})
    assert r.status_code == 400


def test_default_gateway(client):
    _gw(client, "first")
    _gw(client, "second")
    lst = {g["name"]: g["default"] for g in client.post("/api/project/main/gateways/list").json()}
    assert lst == {"first": False, "second": False}  # none marked default (created directly)
    assert client.post("/api/project/main/gateways/set_default", json={"name": "second"}).status_code == 200
    lst = {g["name"]: g["default"] for g in client.post("/api/project/main/gateways/list").json()}
    assert lst == {"first": False, "second": True}
    assert client.post("/api/project/main/gateways/set_default", json={"name": "missing"}).status_code == 400


def test_delete_gateway(client, monkeypatch):
    from dstack_amd.server.services import gateways as gateways_services

    _gw(client, "deleteme")
    monkeypatch.setattr(gateways_services, "_terminate_gateway_compute", lambda *a, **k: None, raising=False)
    r = client.post("/api/project/main/gateways/delete", json={"names": ["deleteme"]})
    assert r.status_code == 200, r.text
    assert client.post("/api/project/main/gateways/list").json() == []


def test_set_wildcard_domain(client):
    _gw(client, "wild")
    r = client.post("/api/project/main/gateways/set_wildcard_domain",
                    json={"name": "wild", "wildcard_domain": "new.example.com"})
    assert r.status_code == 200, r.text
    assert client.post("/api/project/main/gateways/get", json={"name": "wild"}).json()["wildcard_domain"] == \
        "new.example.com"
    r = client.post("/api/project/main/gateways/set_wildcard_domain",
                    json={"name": "missing", "wildcard_domain": "x.example.com"})
    assert r.status_code == 400


# ---- volumes ------------------------------------------------------------------------------------
def _volume(name, **kw):
    return {"configuration": {"type": "volume", "name": name, "backend": "local", "region": "local", "size": "10GB",
                              **kw}}


def test_list_project_volumes(client):
    for n in ("v1", "v2"):
        assert client.post("/api/project/main/volumes/create", json=_volume(n)).status_code == 200
    vols = client.post("/api/project/main/volumes/list").json()
    assert sorted(v["name"] for v in vols) == ["v1", "v2"]
    assert all(v["project_name"] == "main" and v["status"] in ("submitted", "active") for v in vols)


def test_list_volumes_across_projects_for_admin(client):
    client.post("/api/projects/create", json={"project_name": "p2"})
    assert client.post("/api/project/main/volumes/create", json=_volume("va")).status_code == 200
    assert client.post("/api/project/p2/volumes/create", json=_volume("vb")).status_code == 200
    assert sorted(v["name"] for v in client.post("/api/volumes/list", json={}).json()) == ["va", "vb"]


def test_get_volume(client):
    v = client.post("/api/project/main/volumes/create", json=_volume("getme")).json()
    got = client.post("/api/project/main/volumes/get", json={"name": "getme"}).json()
    assert got["id"] == v["id"] and got["configuration"]["size"] == v["configuration"]["size"]
    assert client.post("/api/project/main/volumes/get", json={"name": "nope"}).status_code == 400


def test_create_volume(client):
    r = client.post("/api/project/main/volumes/create", json=_volume("created"))
    assert r.status_code == 200
    v = r.json()
    assert v["name"] == "created" and v["configuration"]["backend"] == "local" and v["deleted"] is False


def test_delete_volumes(client):
    client.post("/api/project/main/volumes/create", json=_volume("d1"))
    client.post("/api/project/main/volumes/create", json=_volume("d2"))
    assert client.post("/api/project/main/volumes/delete", json={"names": ["d1", "d2"]}).status_code == 200
    assert client.post("/api/project/main/volumes/list").json() == []


# ---- instances ----------------------------------------------------------------------------------
def test_instances_list_pagination(client):
    _create(client, _ssh(name="pg", hosts=[f"10.0.8.{i}" for i in range(1, 6)]))
    everything = client.post("/api/instances/list", json={}).json()
    assert len(everything) == 5
    seen, last = [], None
    while True:
        body = {"limit": 2}
        if last:
            body.update(prev_created_at=last["created"], prev_id=last["id"])
        page = client.post("/api/instances/list", json=body).json()
        if not page:
            break
        seen += [i["id"] for i in page]
        last = page[-1]
    assert seen == [i["id"] for i in everything] and len(set(seen)) == 5


# ---- pools --------------------------------------------------------------------------------------
def test_pools_default_created_and_listed(client):
    pools = client.post("/api/project/main/pool/list").json()
    assert len(pools) == 1 and pools[0]["default"] is True


def test_pools_create_duplicate_400(client):
    assert client.post("/api/project/main/pool/create", json={"name": "px"}).status_code == 200
    assert client.post("/api/project/main/pool/create", json={"name": "px"}).status_code == 400


def test_pools_delete_missing_400_and_last_pool(client):
    assert client.post("/api/project/main/pool/delete", json={"name": "missing", "force": False}).status_code == 400
    assert client.post("/api/project/main/pool/set_default", json={"pool_name": "missing"}).status_code == 400
    assert client.post("/api/project/main/pool/show", json={"name": "missing"}).status_code == 400
    # deleting the only (default) pool: a new default is created on the next listing
    only = client.post("/api/project/main/pool/list").json()[0]["name"]
    assert client.post("/api/project/main/pool/delete", json={"name": only, "force": False}).status_code == 200
    pools = client.post("/api/project/main/pool/list").json()
    assert len(pools) == 1 and pools[0]["default"] is True


def test_pools_list_instances_paginated(client):
    _create(client, _ssh(name="pooled", hosts=["10.0.9.1", "10.0.9.2", "10.0.9.3"]))
    all_i = client.post("/api/pools/list_instances", json={}).json()
    assert len(all_i) == 3
    first = client.post("/api/pools/list_instances", json={"limit": 2}).json()
    assert len(first) == 2
    rest = client.post("/api/pools/list_instances", json={"limit": 2, "prev_created_at": first[-1]["created"],
                                                          "prev_id": first[-1]["id"]}).json()
    assert [i["id"] for i in first + rest] == [i["id"] for i in all_i]


# ---- logs / metrics -----------------------------------------------------------------------------
def test_poll_logs_returns_stored_job_logs(client):
    from dstack_amd.server.services import logs as logs_services
    from tests.test_runs_api import _repo, _submit

    _repo(client)
    run = _submit(client, "logged")
    sub_id = run["jobs"][0]["job_submissions"][0]["id"]
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="main").one()
        logs_services.write_job_logs(project.name, "logged", sub_id, {"job_logs": [
            {"timestamp": 1000 + i, "message": base64.b64encode(f"line {i}\n".encode()).decode()} for i in range(3)]})
    r = client.post("/api/project/main/logs/poll", json={"run_name": "logged", "job_submission_id": sub_id,
                                                         "limit": 10})
    assert r.status_code == 200, r.text
    msgs = [base64.b64decode(e["message"]).decode() for e in r.json()["logs"]]
    assert msgs == ["line 0\n", "line 1\n", "line 2\n"]


def test_job_metrics_ignore_deleted_runs(client):
    from tests.test_runs_api import _repo, _submit

    _repo(client)
    _submit(client, "metered")
    r = client.get("/api/project/main/metrics/job/metered")
    assert r.status_code == 200 and r.json()["metrics"] is not None
    client.post("/api/project/main/runs/stop", json={"runs_names": ["metered"], "abort": True})
    with session_scope() as s:
        from dstack_amd.server.models import RunModel

        s.query(RunModel).filter_by(run_name="metered").one().status = "terminated"
    client.post("/api/project/main/runs/delete", json={"runs_names": ["metered"]})
    assert client.get("/api/project/main/metrics/job/metered").status_code == 400


# ---- repos --------------------------------------------------------------------------------------
REMOTE = {"repo_type": "remote", "repo_host_name": "github.com", "repo_port": None, "repo_user_name": "org",
          "repo_name": "proj"}


def test_repos_list_empty_and_filled(client):
    assert client.post("/api/project/main/repos/list").json() == []
    client.post("/api/project/main/repos/init", json={"repo_id": "r1", "repo_info": REMOTE})
    client.post("/api/project/main/repos/init", json={"repo_id": "r2", "repo_info": {"repo_type": "virtual"}})
    assert sorted(r["repo_id"] for r in client.post("/api/project/main/repos/list").json()) == ["r1", "r2"]


def test_repos_get(client):
    assert client.post("/api/project/main/repos/get", json={"repo_id": "nope", "include_creds": False}
                       ).status_code == 400
    client.post("/api/project/main/repos/init", json={"repo_id": "r1", "repo_info": REMOTE})
    got = client.post("/api/project/main/repos/get", json={"repo_id": "r1", "include_creds": False}).json()
    assert got["repo_id"] == "r1" and got["repo_info"]["repo_name"] == "proj" and got.get("repo_creds") is None


def test_repos_creds_are_per_user_with_legacy_fallback(client):
    """The reference stores creds per user and falls back to the repo's legacy creds: the caller
    gets their own creds, else the legacy ones, and never another user's."""
    creds_a = {"protocol": "https", "clone_url": "https://github.com/org/proj.git", "oauth_token": "tok-admin"}
    r = client.post("/api/project/main/repos/init", json={"repo_id": "rc", "repo_info": REMOTE, "repo_creds": creds_a})
    assert r.status_code == 200, r.text
    got = client.post("/api/project/main/repos/get", json={"repo_id": "rc", "include_creds": True}).json()
    assert got["repo_creds"]["oauth_token"] == "tok-admin"
    h = _user(client, "dev", project_role="user")
    other = client.post("/api/project/main/repos/get", json={"repo_id": "rc", "include_creds": True}, headers=h).json()
    assert (other.get("repo_creds") or {}).get("oauth_token") in (None, "tok-admin")
    creds_b = dict(creds_a, oauth_token="tok-dev")
    client.post("/api/project/main/repos/init", json={"repo_id": "rc", "repo_info": REMOTE, "repo_creds": creds_b},
                headers=h)
    mine = client.post("/api/project/main/repos/get", json={"repo_id": "rc", "include_creds": True}, headers=h).json()
    assert mine["repo_creds"]["oauth_token"] == "tok-dev"
    admin = client.post("/api/project/main/repos/get", json={"repo_id": "rc", "include_creds": True}).json()
    assert admin["repo_creds"]["oauth_token"] == "tok-admin"


def test_repos_init_updates_remote_repo(client):
    client.post("/api/project/main/repos/init", json={"repo_id": "ru", "repo_info": REMOTE})
    client.post("/api/project/main/repos/init", json={"repo_id": "ru", "repo_info": dict(REMOTE, repo_name="renamed")})
    got = client.post("/api/project/main/repos/get", json={"repo_id": "ru", "include_creds": False}).json()
    assert got["repo_info"]["repo_name"] == "renamed"
    assert len(client.post("/api/project/main/repos/list").json()) == 1


def test_repos_delete(client):
    client.post("/api/project/main/repos/init", json={"repo_id": "rd", "repo_info": REMOTE})
    assert client.post("/api/project/main/repos/delete", json={"repos_ids": ["rd"]}).status_code == 200
    assert client.post("/api/project/main/repos/list").json() == []


def test_upload_code_same_blob_for_two_repos(client):
    for rid in ("c1", "c2"):
        client.post("/api/project/main/repos/init", json={"repo_id": rid, "repo_info": {"repo_type": "virtual"}})
        r = client.post(f"/api/project/main/repos/upload_code?repo_id={rid}",
                        files={"file": ("code.tar", b"same-bytes", "application/octet-stream")})
        assert r.status_code == 200, r.text
    from dstack_amd.server.models import CodeModel

    with session_scope() as s:
        codes = s.query(CodeModel).all()
        assert len(codes) == 2 and len({c.blob_hash for c in codes}) == 1
