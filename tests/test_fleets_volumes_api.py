"""Fleets, instances, volumes and gateways REST APIs (reference: ``src/tests/_internal/server/routers/
test_{fleets,instances,volumes,gateways}.py``): SSH-fleet validation, cloud fleets with ``nodes``
ranges and cluster placement, deleting fleets / single instances while in use, instance listing
filters, volume and gateway CRUD with the backend capability checks."""

from __future__ import annotations

import pytest

from dstack_amd.core.models.instances import InstanceStatus
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import FleetModel, InstanceModel

KEY = {"public": "ssh-ed25519 AAAA", "private": "-----BEGIN OPENSSH PRIVATE KEY-----\nx\n"
                                               "-----END OPENSSH PRIVATE KEY-----\n"}


def _fleet(conf: dict) -> dict:
    return {"spec": {"configuration": {"type": "fleet", **conf}, "profile": {"name": "default"}}}


def _ssh(name="onprem", hosts=("10.0.0.1",), **kw):
    sc = {"user": "ubuntu", "ssh_key": KEY, "hosts": list(hosts)}
    sc.update(kw)
    return _fleet({"name": name, "ssh_config": sc})


def _create(client, body):
    r = client.post("/api/project/main/fleets/create", json=body)
    assert r.status_code == 200, r.text
    return r.json()


# ---- SSH fleets -----------------------------------------------------------------------------
def test_ssh_fleet_instances_per_host_with_blocks(client):
    fleet = _create(client, _ssh(hosts=["10.0.0.1", {"hostname": "10.0.0.2", "blocks": 8, "port": 2222}]))
    insts = sorted(fleet["instances"], key=lambda i: i["instance_num"])
    assert [i["instance_num"] for i in insts] == [0, 1]
    assert all(i["status"] == "pending" and i["backend"] == "remote" for i in insts)
    with session_scope() as s:
        rows = {i.instance_num: i for i in s.query(InstanceModel)}
        assert rows[1].total_blocks == 8 and rows[0].total_blocks == 1
        assert '"port":2222' in rows[1].remote_connection_info.replace(" ", "")
        assert rows[0].termination_idle_time == -1  # SSH hosts are never idle-terminated


@pytest.mark.parametrize("body,msg", [
    (_ssh(ssh_key=None), "No ssh key"),
    (_ssh(user=None), "No ssh user"),
    (_ssh(ssh_key={"public": "x", "private": "not a key"}), "Unsupported key type"),
    (_ssh(ssh_key={"public": "x", "private": "-----BEGIN RSA PRIVATE KEY-----\nProc-Type: 4,ENCRYPTED\n"}),
     "Unsupported key type"),
    (_ssh(hosts=[{"hostname": "10.0.0.1", "internal_ip": "192.168.0.1"}, "10.0.0.2"]), "internal_ip must be"),
    (_ssh(hosts=[{"hostname": "10.0.0.1", "internal_ip": "192.168.0.1"}], network="192.168.0.0/24"),
     "mutually exclusive"),
    (_fleet({"name": "empty"}), "nodes"),
    (_ssh(name="Bad_Name"), "Fleet name"),
])
def test_invalid_fleet_specs_rejected(client, body, msg):
    r = client.post("/api/project/main/fleets/create", json=body)
    assert r.status_code in (400, 422), r.text  # 422: rejected by the configuration model itself
    assert msg in r.text


def test_server_never_reads_identity_file_path(client, tmp_path):
    """An identity_file path alone (no key contents) is rejected: the CLI reads the file."""
    secret = tmp_path / "server-secret"
    secret.write_text("-----BEGIN OPENSSH PRIVATE KEY-----\nserver\n-----END OPENSSH PRIVATE KEY-----\n")
    body = _ssh(ssh_key=None, identity_file=str(secret))
    assert client.post("/api/project/main/fleets/create", json=body).status_code == 400


def test_cli_resolves_identity_files(tmp_path):
    from dstack_amd.cli.configurators import _resolve_ssh_keys
    from dstack_amd.core.models.fleets import FleetConfiguration

    k = tmp_path / "id_ed25519"
    k.write_text(KEY["private"])
    (tmp_path / "id_ed25519.pub").write_text("ssh-ed25519 AAAA me\n")
    conf = FleetConfiguration.model_validate({"type": "fleet", "name": "f", "ssh_config": {
        "user": "u", "identity_file": str(k), "hosts": ["h1", {"hostname": "h2", "identity_file": str(k)}]}})
    _resolve_ssh_keys(conf)
    assert conf.ssh_config.ssh_key.private == KEY["private"]
    assert conf.ssh_config.ssh_key.public == "ssh-ed25519 AAAA me"
    assert conf.ssh_config.hosts[1].ssh_key.private == KEY["private"]


def test_duplicate_fleet_name(client):
    _create(client, _ssh(name="dup"))
    assert client.post("/api/project/main/fleets/create", json=_ssh(name="dup")).status_code == 400


# ---- cloud fleets ---------------------------------------------------------------------------
def test_cloud_fleet_nodes_range_creates_min_nodes(client):
    fleet = _create(client, _fleet({"name": "cloud", "nodes": "2..4", "placement": "cluster",
                                    "resources": {"gpu": "MI355X:8"}, "idle_duration": "1h"}))
    assert len(fleet["instances"]) == 2
    with session_scope() as s:
        rows = list(s.query(InstanceModel).filter_by(status=InstanceStatus.PENDING.value))
        assert {r.termination_idle_time for r in rows} == {3600}
        assert all('"placement": "cluster"' in r.backend_data for r in rows)


def test_fleet_plan_lists_offers_of_configured_backends(client):
    client.post("/api/project/main/backends/create", json={"type": "vultr", "creds": {"type": "api_key",
                                                                                      "api_key": "k"}})
    plan = client.post("/api/project/main/fleets/get_plan", json=_fleet(
        {"name": "p", "nodes": 1, "resources": {"gpu": "MI355X:8"}})).json()
    assert plan["total_offers"] >= 1
    assert all(o["instance"]["resources"]["gpus"][0]["name"] == "MI355X" for o in plan["offers"])
    assert plan["current_resource"] is None


# ---- deleting fleets and instances -----------------------------------------------------------
def test_delete_fleet_in_use_rejected_then_allowed(client):
    fleet = _create(client, _ssh(name="busy", hosts=["10.0.0.1", "10.0.0.2"]))
    with session_scope() as s:
        for i in s.query(InstanceModel):
            i.status = InstanceStatus.BUSY.value if i.instance_num == 0 else InstanceStatus.IDLE.value
    r = client.post("/api/project/main/fleets/delete", json={"names": ["busy"]})
    assert r.status_code == 400 and "busy" in r.text
    # an idle instance of the fleet can go on its own; the busy one cannot
    r = client.post("/api/project/main/fleets/delete_instances", json={"name": "busy", "instance_nums": [1]})
    assert r.status_code == 200, r.text
    r = client.post("/api/project/main/fleets/delete_instances", json={"name": "busy", "instance_nums": [0]})
    assert r.status_code == 400
    with session_scope() as s:
        st = {i.instance_num: i.status for i in s.query(InstanceModel)}
        assert st == {0: InstanceStatus.BUSY.value, 1: InstanceStatus.TERMINATING.value}
        s.query(InstanceModel).filter_by(instance_num=0).one().status = InstanceStatus.IDLE.value
    assert client.post("/api/project/main/fleets/delete", json={"names": ["busy"]}).status_code == 200
    with session_scope() as s:
        assert s.query(FleetModel).filter_by(name="busy").one().status == "terminating"
    assert fleet["name"] == "busy"
    assert client.post("/api/project/main/fleets/delete", json={"names": ["nope"]}).status_code == 400


def test_empty_fleet_deleted_by_reconciler(client):
    from dstack_amd.server.background.tasks import process_fleets as pf

    _create(client, _ssh(name="gone"))
    client.post("/api/project/main/fleets/delete", json={"names": ["gone"]})
    with session_scope() as s:
        for i in s.query(InstanceModel):
            i.status = InstanceStatus.TERMINATED.value
            i.deleted = True
    with session_scope() as s:
        fid = s.query(FleetModel).filter_by(name="gone").one().id
        pf._process_fleet(s, fid)
    with session_scope() as s:
        f = s.get(FleetModel, fid)
        assert f.deleted and f.status == "terminated"
    assert client.post("/api/project/main/fleets/list").json() == []


# ---- instances listing -------------------------------------------------------------------------
def test_instances_list_filters(client):
    a = _create(client, _ssh(name="fa", hosts=["10.0.1.1"]))
    _create(client, _ssh(name="fb", hosts=["10.0.1.2", "10.0.1.3"]))
    assert len(client.post("/api/instances/list", json={}).json()) == 3
    only_a = client.post("/api/instances/list", json={"fleet_ids": [a["id"]]}).json()
    assert [i["fleet_name"] for i in only_a] == ["fa"]
    assert client.post("/api/instances/list", json={"project_names": ["other"]}).json() == []
    with session_scope() as s:
        for i in s.query(InstanceModel).filter(InstanceModel.name.like("fb-%")):
            i.status = InstanceStatus.TERMINATED.value
    active = client.post("/api/instances/list", json={"only_active": True}).json()
    assert [i["fleet_name"] for i in active] == ["fa"]


# ---- volumes ------------------------------------------------------------------------------------
def _volume(name="vol1", backend="local", region="local", size="100GB", **kw):
    return {"configuration": {"type": "volume", "name": name, "backend": backend, "region": region, "size": size,
                              **kw}}


def test_volume_crud_and_capability_check(client):
    r = client.post("/api/project/main/volumes/create", json=_volume())
    assert r.status_code == 200, r.text
    v = r.json()
    assert v["name"] == "vol1" and v["configuration"]["backend"] == "local"
    assert client.post("/api/project/main/volumes/create", json=_volume()).status_code == 400  # exists
    r = client.post("/api/project/main/volumes/create", json=_volume("vol2", backend="vultr", region="ewr"))
    assert r.status_code == 400 and "does not support volumes" in r.text
    got = client.post("/api/project/main/volumes/get", json={"name": "vol1"}).json()
    assert got["id"] == v["id"]
    assert [x["name"] for x in client.post("/api/volumes/list", json={}).json()] == ["vol1"]
    assert client.post("/api/project/main/volumes/delete", json={"names": ["vol1"]}).status_code == 200
    assert client.post("/api/project/main/volumes/delete", json={"names": ["nope"]}).status_code == 400


def test_attached_volume_cannot_be_deleted(client):
    from dstack_amd.server.models import VolumeModel

    client.post("/api/project/main/volumes/create", json=_volume("data"))
    _create(client, _ssh(name="host"))
    with session_scope() as s:
        vol = s.query(VolumeModel).filter_by(name="data").one()
        inst = s.query(InstanceModel).one()
        vol.instances.append(inst)
    r = client.post("/api/project/main/volumes/delete", json={"names": ["data"]})
    assert r.status_code == 400 and "attached" in r.text


def test_volume_plan(client):
    plan = client.post("/api/project/main/volumes/get_plan", json={"spec": {"configuration": _volume()[
        "configuration"]}})
    assert plan.status_code == 200, plan.text
    assert plan.json()["spec"]["configuration"]["name"] == "vol1"


# ---- gateways -----------------------------------------------------------------------------------
def test_gateway_capability_and_duplicates(client):
    conf = {"configuration": {"type": "gateway", "name": "gw", "backend": "vultr", "region": "ewr",
                              "domain": "example.com"}}
    r = client.post("/api/project/main/gateways/create", json=conf)
    assert r.status_code == 400 and "does not support gateways" in r.text
    conf["configuration"].update(backend="aws", region="us-east-1")
    r = client.post("/api/project/main/gateways/create", json=conf)
    assert r.status_code == 400 and "not configured" in r.text
    assert client.post("/api/project/main/gateways/delete", json={"names": ["gw"]}).status_code == 400
    assert client.post("/api/project/main/gateways/set_default", json={"name": "gw"}).status_code == 400


def test_delete_fleet_refuses_instance_with_unfinished_job(client):
    """A PROVISIONING instance created for a just-submitted job is in use even though it is not
    BUSY yet: the fleet delete must not terminate it under the job."""
    from dstack_amd.server.models import JobModel

    from tests.test_reconcilers import _job, _submit

    _create(client, _ssh(name="prov", hosts=["10.0.0.9"]))
    with session_scope() as s:
        rid = _submit(s, {"type": "task", "commands": ["x"]}, name="r-prov")
        inst = s.query(InstanceModel).one()
        inst.status = InstanceStatus.PROVISIONING.value
        j = _job(s, rid)
        j.instance_id = inst.id
        j.status = "provisioning"
    r = client.post("/api/project/main/fleets/delete", json={"names": ["prov"]})
    assert r.status_code == 400 and "busy" in r.text
    with session_scope() as s:
        assert s.query(InstanceModel).one().status == InstanceStatus.PROVISIONING.value
        s.query(JobModel).one().status = "done"
    assert client.post("/api/project/main/fleets/delete", json={"names": ["prov"]}).status_code == 200


def test_lock_wait_timeout_is_a_409_not_a_500(client):
    """A request that waits too long for a row a reconciler holds gets 409 'retry', not a 500."""
    from dstack_amd.server.services import fleets as fleets_services
    from dstack_amd.server.services.locking import lockset

    _create(client, _ssh(name="held", hosts=["10.0.0.7"]))
    with session_scope() as s:
        fid = s.query(FleetModel).filter_by(name="held").one().id
    orig = fleets_services._held

    def short_held(fleets, instances, timeout=60.0):
        return orig(fleets, instances, timeout=0.2)

    lockset("fleets").add_all_or_nothing([fid])  # a background pass holds the fleet
    try:
        fleets_services._held = short_held
        r = client.post("/api/project/main/fleets/delete", json={"names": ["held"]})
    finally:
        fleets_services._held = orig
        lockset("fleets").remove_many([fid])
    assert r.status_code == 409, r.text
    assert r.json()["detail"][0]["code"] == "resource_busy"
