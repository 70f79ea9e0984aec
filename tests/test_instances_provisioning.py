"""Cloud-fleet instance provisioning in ``process_instances`` (reference: ``src/tests/_internal/server/
background/tasks/test_process_instances.py``): ``placement: cluster`` fleets provision the first
node, then the rest in its backend/region/availability zone inside one placement group; no-capacity
retries every minute until ``retry.duration`` runs out; without retry the instance is terminated;
``blocks`` split a new instance's GPUs; offers from backends that cannot create instances are
skipped."""

from __future__ import annotations

import json
from datetime import timedelta
from typing import List
from unittest import mock

import pytest

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import (
    Disk,
    Gpu,
    InstanceAvailability,
    InstanceOfferWithAvailability,
    InstanceStatus,
    InstanceType,
    Resources,
)
from dstack_amd.core.models.placement import PlacementGroupProvisioningData
from dstack_amd.core.models.runs import JobProvisioningData
from dstack_amd.server.background.tasks import process_instances as pi
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import FleetModel, InstanceModel, PlacementGroupModel, ProjectModel, UserModel
from dstack_amd.server.services import fleets as fleets_services
from dstack_amd.utils.common import get_current_datetime


def _offer(backend=BackendType.AWS, region="us-east-1", gpus=8, price=10.0):
    it = InstanceType(name="p-mi355x", resources=Resources(cpus=128, memory_mib=2048 * 1024,
                                                           gpus=[Gpu(name="MI355X", memory_mib=288 * 1024)] * gpus,
                                                           disk=Disk(size_mib=1024 * 1024)))
    return InstanceOfferWithAvailability(backend=backend, instance=it, region=region, price=price,
                                         availability=InstanceAvailability.AVAILABLE)


class FakeCompute:
    def __init__(self, fail: bool = False):
        self.created: List[tuple] = []
        self.pgs: List[str] = []
        self.fail = fail

    def create_instance(self, offer, cfg):
        if self.fail:
            raise RuntimeError("InsufficientInstanceCapacity")
        self.created.append((offer.backend, offer.region, cfg.availability_zone, cfg.placement_group_name))
        return JobProvisioningData(backend=offer.backend, instance_type=offer.instance, instance_id=f"i-{len(self.created)}",
                                   hostname=None, internal_ip=None, region=offer.region, price=offer.price,
                                   username="ubuntu", ssh_port=22, dockerized=True,
                                   availability_zone=f"{offer.region}a")

    def create_placement_group(self, pg):
        self.pgs.append(pg.name)
        return PlacementGroupProvisioningData(backend=pg.configuration.backend)


def _fleet(s, conf: dict):
    from dstack_amd.core.models.fleets import FleetSpec

    project = s.query(ProjectModel).filter_by(name="main").one()
    user = s.query(UserModel).filter_by(name="admin").one()
    spec = FleetSpec.model_validate({"configuration": {"type": "fleet", **conf}, "profile": {"name": "default"}})
    return fleets_services.create_fleet(s, project, user, spec)


def _instances(s, fleet_name):
    f = s.query(FleetModel).filter_by(name=fleet_name).one()
    return sorted(f.instances, key=lambda i: i.instance_num)


def _process(iid, offers_fn, at=None):
    patches = [mock.patch.object(pi.offers_services, "get_offers_by_requirements", side_effect=offers_fn)]
    if at is not None:
        patches.append(mock.patch.object(pi, "get_current_datetime", return_value=at))
    for p in patches:
        p.start()
    try:
        with session_scope() as s:
            pi._process_instance(s, iid)
    finally:
        for p in patches:
            p.stop()


def test_cluster_fleet_follows_first_node(db):
    comp = FakeCompute()
    calls = []

    def offers(s, project, profile, req, **kw):
        calls.append(kw)
        mj = kw.get("master_job_provisioning_data")
        if mj is not None:
            return [(comp, _offer(mj.backend, mj.region))]
        return [(comp, _offer(BackendType.AWS, "us-west-2", price=9.0)), (comp, _offer(BackendType.AWS, "us-east-1"))]

    with session_scope() as s:
        _fleet(s, {"name": "clu", "nodes": 3, "placement": "cluster", "resources": {"gpu": "MI355X:8"}})
        ids = [i.id for i in _instances(s, "clu")]
    _process(ids[1], offers)  # a follower before the first node: waits, no offers queried
    assert calls == [] and comp.created == []
    _process(ids[0], offers)
    assert comp.created[0][:2] == (BackendType.AWS, "us-west-2") and calls[0]["multinode"]
    for iid in ids[1:]:
        _process(iid, offers)
    assert [c[:3] for c in comp.created[1:]] == [(BackendType.AWS, "us-west-2", "us-west-2a")] * 2
    # one placement group for the fleet in that backend/region, used by every node
    assert len(comp.pgs) == 1 and {c[3] for c in comp.created} == {comp.pgs[0]}
    with session_scope() as s:
        assert s.query(PlacementGroupModel).count() == 1
        assert {i.status for i in _instances(s, "clu")} == {InstanceStatus.PROVISIONING.value}


def test_no_capacity_retried_every_minute_until_duration(db):
    comp = FakeCompute(fail=True)
    with session_scope() as s:
        _fleet(s, {"name": "retry", "nodes": 1, "retry": {"on_events": ["no-capacity"], "duration": "10m"}})
        (inst,) = _instances(s, "retry")
        iid, created = inst.id, inst.created_at
    offers = lambda *a, **k: [(comp, _offer())]  # noqa: E731
    _process(iid, offers)
    with session_scope() as s:
        i = s.get(InstanceModel, iid)
        assert i.status == InstanceStatus.PENDING.value and i.last_retry_at is not None
        assert i.termination_reason == "all offers failed"
    # within the minute: not retried; after it: retried
    with mock.patch.object(comp, "create_instance", side_effect=RuntimeError("x")) as ci:
        _process(iid, offers, at=created + timedelta(seconds=20))
        assert ci.call_count == 0
        _process(iid, offers, at=created + timedelta(minutes=2))
        assert ci.call_count == 1
    _process(iid, offers, at=created + timedelta(minutes=11))
    with session_scope() as s:
        i = s.get(InstanceModel, iid)
        assert i.status == InstanceStatus.TERMINATED.value and i.termination_reason == "Retry duration expired"


def test_no_offers_without_retry_terminates(db):
    with session_scope() as s:
        _fleet(s, {"name": "noretry", "nodes": 1})
        (inst,) = _instances(s, "noretry")
        iid = inst.id
    _process(iid, lambda *a, **k: [])
    with session_scope() as s:
        i = s.get(InstanceModel, iid)
        assert i.status == InstanceStatus.TERMINATED.value and "no offers" in i.termination_reason


@pytest.mark.parametrize("blocks,expect", [(1, 1), (4, 4), ("auto", 8)])
def test_fleet_blocks_split_new_instance(db, blocks, expect):
    comp = FakeCompute()
    seen = {}

    def offers(s, project, profile, req, **kw):
        seen["blocks"] = kw.get("blocks")
        return [(comp, _offer())]

    with session_scope() as s:
        _fleet(s, {"name": "blk", "nodes": 1, "blocks": blocks})
        (inst,) = _instances(s, "blk")
        iid = inst.id
    _process(iid, offers)
    assert seen["blocks"] == blocks
    with session_scope() as s:
        assert s.get(InstanceModel, iid).total_blocks == expect


def test_offers_of_backends_without_create_instance_skipped(db):
    comp = FakeCompute()
    with session_scope() as s:
        _fleet(s, {"name": "skip", "nodes": 1})
        (inst,) = _instances(s, "skip")
        iid = inst.id
    _process(iid, lambda *a, **k: [(comp, _offer(BackendType.RUNPOD, "EU-RO-1", gpus=1, price=1.0)),
                                   (comp, _offer(BackendType.VULTR, "ewr"))])
    assert [c[0] for c in comp.created] == [BackendType.VULTR]


def test_blocks_offer_helper_keeps_int_blocks():
    from dstack_amd.server.services.offers import _with_blocks

    assert _with_blocks(_offer(gpus=8), 2).total_blocks == 2
    assert _with_blocks(_offer(gpus=8), "auto").total_blocks == 8
    assert _with_blocks(_offer(gpus=0), "auto").total_blocks == 128  # CPU host: one block per CPU


@pytest.mark.parametrize("cpus,gpus,requested,expected", [
    (32, 8, 1, 1), (32, 8, 2, 2), (32, 8, 4, 4), (32, 8, "auto", 8), (4, 8, "auto", 4), (8, 8, "auto", 8),
    (32, 0, 1, 1), (32, 0, 2, 2), (32, 0, 4, 4), (32, 0, "auto", 32),
], ids=["gpu-no-blocks", "gpu-4-per-block", "gpu-2-per-block", "gpu-auto-max-gpu", "gpu-auto-max-cpu",
        "gpu-auto-max-cpu-and-gpu", "cpu-no-blocks", "cpu-16-per-block", "cpu-8-per-block", "cpu-auto-max-cpu"])
def test_block_counts_for_created_and_ssh_instances(cpus, gpus, requested, expected):
    """Reference ``TestCreateInstance`` / ``TestAddSSHInstance`` block tables: a cloud offer and an
    SSH host get the same block count for the same shape."""
    from dstack_amd.core.backends.remote import split_blocks
    from dstack_amd.core.models.instances import GpuDevice, HostTopology
    from dstack_amd.server.services.offers import _with_blocks

    o = _offer(gpus=gpus)
    o.instance.resources.cpus = cpus
    assert _with_blocks(o, requested).total_blocks == expected
    topo = HostTopology(gpus=[GpuDevice(index=i, name="MI355X", memory_mib=288 * 1024) for i in range(gpus)])
    assert split_blocks(topo, requested, cpus) == expected


def test_fleet_backend_data_records_placement(db):
    with session_scope() as s:
        _fleet(s, {"name": "bd", "nodes": 2, "placement": "cluster"})
        assert all(json.loads(i.backend_data)["placement"] == "cluster" for i in _instances(s, "bd"))
    _ = get_current_datetime


# ---- SSH-fleet deploys across server replicas ----------------------------------------------------
HOST_INFO = {"cpus": 128, "memory": 2 << 40, "disk_size": 10 << 40, "addresses": ["10.0.0.5/eth0"],
             "topology": {"gpus": [{"index": i, "name": "MI355X", "memory_mib": 288 * 1024} for i in range(8)],
                          "xgmi": [[int(i != j) for j in range(8)] for i in range(8)], "numa": {}, "nics": []}}


def _remote_instance(s):
    from dstack_amd.core.models.instances import SSHKey
    from dstack_amd.server.services import pools as pools_services

    project = s.query(ProjectModel).filter_by(name="main").one()
    inst = pools_services.add_remote(s, project, None, "h5", None, None, "10.0.0.5", 22, "ubuntu",
                                     [SSHKey(public="ssh-ed25519 AAAA", private="k")])
    return inst.id


def test_ssh_deploy_leased_once_across_replicas(db, monkeypatch):
    """Two server replicas on one database, each with its own in-process deploy futures: the replica
    that starts a host's deploy leases the instance row, the other skips it (even past the 30 s
    retry gate), only the owner applies the result, and an expired lease of a dead replica is taken
    over (reference: the instance lock across the deploy, process_instances.py:210-377)."""
    import threading

    from dstack_amd.server import settings

    with session_scope() as s:
        iid = _remote_instance(s)
    gate, calls = threading.Event(), []

    def fake_deploy(rci, pub, key, **kw):
        calls.append(rci.host)
        assert gate.wait(10)
        return HOST_INFO

    monkeypatch.setattr(pi, "deploy_ssh_instance", fake_deploy)

    def as_replica(name, deploys):
        monkeypatch.setattr(settings, "SERVER_REPLICA_ID", name)
        monkeypatch.setattr(pi, "_deploys", deploys)

    a, b = {}, {}
    as_replica("A", a)
    with session_scope() as s:
        pi._add_remote(s, s.get(InstanceModel, iid))
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.deploy_owner == "A" and inst.status == InstanceStatus.PENDING.value
        inst.last_retry_at = get_current_datetime() - timedelta(minutes=5)  # past the retry gate
    as_replica("B", b)
    for _ in range(3):
        with session_scope() as s:
            pi._add_remote(s, s.get(InstanceModel, iid))
    assert calls == ["10.0.0.5"] and not b  # B never started a second deploy
    gate.set()
    a[iid].result(timeout=10)
    with session_scope() as s:  # B sees the finished deploy's instance still leased: hands off
        pi._add_remote(s, s.get(InstanceModel, iid))
        assert s.get(InstanceModel, iid).status == InstanceStatus.PENDING.value
    as_replica("A", a)
    with session_scope() as s:
        pi._add_remote(s, s.get(InstanceModel, iid))
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == InstanceStatus.IDLE.value and inst.total_blocks == 1
        assert inst.deploy_owner is None and inst.deploy_started_at is None
    assert len(calls) == 1
    # a replica that died mid-deploy: its lease expires after the deploy deadline, then another
    # replica re-deploys the host
    with session_scope() as s:
        iid2 = _remote_instance_named(s, "10.0.0.6")
        inst = s.get(InstanceModel, iid2)
        inst.deploy_owner = "dead-replica"
        inst.deploy_started_at = get_current_datetime() - pi.DEPLOY_LEASE - timedelta(seconds=1)
    as_replica("B", b)
    with session_scope() as s:
        pi._add_remote(s, s.get(InstanceModel, iid2))
    b[iid2].result(timeout=10)
    assert calls == ["10.0.0.5", "10.0.0.6"]
    with session_scope() as s:
        pi._add_remote(s, s.get(InstanceModel, iid2))
        assert s.get(InstanceModel, iid2).status == InstanceStatus.IDLE.value


def _remote_instance_named(s, host):
    from dstack_amd.core.models.instances import SSHKey
    from dstack_amd.server.services import pools as pools_services

    project = s.query(ProjectModel).filter_by(name="main").one()
    return pools_services.add_remote(s, project, None, None, None, None, host, 22, "ubuntu",
                                     [SSHKey(public="ssh-ed25519 AAAA", private="k")]).id


def test_ssh_instance_terminated_when_provisioning_timeout_expired(db, monkeypatch):
    """(reference ``TestSSHInstanceTerminateProvisionTimeoutExpired``) a pending SSH host that never
    came up within the deadline is given up without another deploy attempt."""
    from datetime import timedelta

    from dstack_amd.server.background.tasks import process_instances as pi

    deploys = []
    monkeypatch.setattr(pi, "deploy_ssh_instance", lambda *a, **k: deploys.append(a) or HOST_INFO)
    with session_scope() as s:
        iid = _remote_instance(s)
        s.get(InstanceModel, iid).created_at = get_current_datetime() - timedelta(days=100)
    with session_scope() as s:
        pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == "terminated" and inst.termination_reason == "Provisioning timeout expired"
    assert deploys == []
