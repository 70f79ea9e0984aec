"""Server services, case by case against the reference's ``server/services/**/test_*.py`` (mapping:
``docs/reference/test-parity.md``): the agent HTTP client (API negotiation, typed errors, task
calls), the RPS autoscaler, registry document parsing and mount-target validation, SSH-fleet host
uniqueness, pool instance naming/conversion, repo credentials, replica scaling, volume attach
checks and per-job volume interpolation."""

from __future__ import annotations

import json
import uuid
from datetime import datetime, timedelta, timezone
from unittest import mock

import httpx
import pytest

from dstack_amd.core.errors import ServerClientError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import InstanceStatus, RemoteConnectionInfo
from dstack_amd.core.models.runs import JobStatus, JobTerminationReason
from dstack_amd.core.models.volumes import InstanceMountPoint, VolumeMountPoint
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import (
    FleetModel,
    InstanceModel,
    JobModel,
    ProjectModel,
    RepoCredsModel,
    RepoModel,
    RunModel,
    UserModel,
    VolumeModel,
)
from dstack_amd.utils.common import get_current_datetime


# ---- runner/test_client.py: ShimClient ----------------------------------------------------------
class _Recorder:
    """An in-process shim: canned answers per (method, path), every request recorded."""

    def __init__(self, routes=None):
        self.routes = dict(routes or {})
        self.requests = []

    def __call__(self, request: httpx.Request) -> httpx.Response:
        self.requests.append(request)
        ans = self.routes.get((request.method, request.url.path))
        if ans is None:
            return httpx.Response(404, json={"error": "not found"})
        status, body = ans
        return httpx.Response(status, json=body)

    def body(self, i):
        return json.loads(self.requests[i].content or b"null")


def _shim(routes=None, version=None, api_version=None):
    from dstack_amd.server.services.runner.client import ShimClient

    rec = _Recorder(routes)
    if version is not None:
        hc = {"service": "dstack-shim", "version": version}
        if api_version is not None:
            hc["api_version"] = api_version
        rec.routes[("GET", "/api/healthcheck")] = (200, hc)
    return ShimClient("http://shim.test", transport=httpx.MockTransport(rec)), rec


@pytest.mark.parametrize("version,expected_shim,expected_api", [
    ("0.0.9", (0, 0, 9), 1),                    # final release before the probe endpoints
    ("0.0.9+build.1", (0, 0, 9), 1),            # local segment ignored
    ("0.1.0", (0, 1, 0), 2),                    # boundary
    ("0.1.0+mi355x", (0, 1, 0), 2),             # what our native shim reports
    ("1494", None, 2),                          # CI build number, not a version: latest
    ("latest", None, 2),
    ("0.0.1-next", None, 2),
    ("0.0.1rc1", None, 2),                      # any non-final version is taken as the latest
])
def test_shim_client_negotiates_api_from_healthcheck(version, expected_shim, expected_api):
    c, rec = _shim(version=version)
    assert not hasattr(c, "_shim_version") and not hasattr(c, "_api_version")
    c._negotiate()
    assert c._shim_version == expected_shim
    assert c._api_version == expected_api
    assert [(r.method, r.url.path) for r in rec.requests] == [("GET", "/api/healthcheck")]


def test_shim_client_explicit_api_version_wins():
    c, _ = _shim(version="0.0.1", api_version=2)
    assert c.api_version == 2


def test_shim_client_raise_for_status_is_typed():
    from dstack_amd.server.services.runner.client import ShimHTTPError

    c, rec = _shim()
    rec.routes[("GET", "/test/path")] = (502, {"error": "upstream"})
    r = c._request("GET", "/test/path")
    with pytest.raises(ShimHTTPError) as ei:
        c._raise_for_status(r)
    assert ei.value.status_code == 502
    assert ei.value.message.startswith("502 Server Error: Bad Gateway")
    assert str(ei.value).startswith("502 Server Error: Bad Gateway")
    assert repr(ei.value) == "ShimHTTPError(502)"


def test_shim_client_healthcheck():
    c, rec = _shim(version="0.1.0")
    assert c.healthcheck() == {"service": "dstack-shim", "version": "0.1.0"}
    assert len(rec.requests) == 1


def test_shim_client_get_task():
    task = {"id": "t1", "status": "running", "termination_reason": "", "termination_message": "",
            "container_name": "horrible-mule-1-0-0", "ports": [{"container": 10022, "host": 32771}]}
    c, rec = _shim({("GET", "/api/tasks/t1"): (200, task)}, version="0.1.0")
    assert c.get_task("t1") == task
    assert c.get_task("missing") is None  # 404 -> None, not an error


def test_shim_client_submit_task_and_conflict():
    c, rec = _shim({("POST", "/api/tasks"): (200, {"id": "t1", "status": "pending"})}, version="0.1.0")
    task = {"id": "t1", "name": "job", "image_name": "rocm/pytorch", "gpus": [0, 1], "privileged": False,
            "volumes": [], "instance_mounts": []}
    assert c.submit_task(task)["status"] == "pending"
    assert rec.requests[-1].method == "POST" and rec.body(-1) == task
    # 409: the task exists already (a resubmit after a lost answer) -> its current state
    rec.routes[("POST", "/api/tasks")] = (409, {"error": "exists"})
    rec.routes[("GET", "/api/tasks/t1")] = (200, {"id": "t1", "status": "running"})
    assert c.submit_task(task) == {"id": "t1", "status": "running"}


def test_shim_client_submit_task_error_status_raises():
    from dstack_amd.server.services.runner.client import ShimHTTPError

    c, _ = _shim({("POST", "/api/tasks"): (400, {"error": "bad image"})}, version="0.1.0")
    with pytest.raises(ShimHTTPError) as ei:
        c.submit_task({"id": "t1"})
    assert ei.value.status_code == 400 and "bad image" in ei.value.message


def test_shim_client_terminate_task():
    c, rec = _shim({("POST", "/api/tasks/t1/terminate"): (200, {})}, version="0.1.0")
    c.terminate_task("t1", "TERMINATED_BY_USER", "stopped from the CLI", timeout=3)
    assert rec.body(-1) == {"termination_reason": "TERMINATED_BY_USER",
                            "termination_message": "stopped from the CLI", "timeout": 3}


def test_shim_client_terminate_task_default_params():
    c, rec = _shim({("POST", "/api/tasks/t1/terminate"): (200, {})}, version="0.1.0")
    c.terminate_task("t1")
    assert rec.body(-1) == {"termination_reason": "", "termination_message": "", "timeout": 10}
    c.terminate_task("gone")  # already removed on the host: not an error


def test_shim_client_remove_task():
    c, rec = _shim({("POST", "/api/tasks/t1/remove"): (200, {})}, version="0.1.0")
    c.remove_task("t1")
    assert (rec.requests[-1].method, rec.requests[-1].url.path) == ("POST", "/api/tasks/t1/remove")


def test_shim_client_api1_shim_has_no_probe_endpoints():
    c, rec = _shim(version="0.0.9")
    assert c.gpu_health() is None and c.start_gpu_probe() == "unavailable"
    assert [r.url.path for r in rec.requests] == ["/api/healthcheck"]  # never asked
    c2, rec2 = _shim({("GET", "/api/gpu_health"): (200, {"state": "done"})}, version="0.1.0")
    assert c2.gpu_health() == {"state": "done"}


@pytest.mark.parametrize("value,expected", [
    ("1.12", (1, 12, 0)), ("1.12.3", (1, 12, 3)), ("1.12.3.1", (1, 12, 3)), ("1.12.3+build.1", (1, 12, 3)),
])
def test_parse_version_valid_final(value, expected):
    from dstack_amd.server.services.runner.client import parse_version

    assert parse_version(value) == expected


@pytest.mark.parametrize("value", [
    "1.12alpha1", "1.12.3rc1", "1.12.3.dev0",   # pre / dev releases
    "1", "1234",                                # major only
    "", "foo", "1.12.3-next.20241231",          # not versions
])
def test_parse_version_non_final_is_none(value):
    from dstack_amd.server.services.runner.client import parse_version

    assert parse_version(value) is None


def test_runner_client_submit_and_pull_over_transport():
    from dstack_amd.server.services.runner.client import RunnerClient

    rec = _Recorder({("POST", "/api/run"): (200, {}),
                     ("GET", "/api/pull"): (200, {"job_states": [], "job_logs": [], "runner_logs": [],
                                                   "last_updated": 5, "has_more": False})})
    rc = RunnerClient("http://runner.test", transport=httpx.MockTransport(rec))
    rc.run_job()
    out = rc.pull(3)
    assert out["last_updated"] == 5
    assert rec.requests[-1].url.params["timestamp"] == "3"


# ---- services/test_autoscalers.py: RPSAutoscaler ------------------------------------------------
_T0 = datetime(2024, 1, 1, tzinfo=timezone.utc)


@pytest.fixture
def frozen_now():
    with mock.patch("dstack_amd.server.services.services.get_current_datetime", return_value=_T0):
        yield _T0


def _rep(active=True, ago=3600):
    from dstack_amd.server.services.services import ReplicaInfo

    return ReplicaInfo(active=active, timestamp=_T0 - timedelta(seconds=ago))


def _rps():
    from dstack_amd.server.services.services import RPSAutoscaler

    return RPSAutoscaler(0, 5, 10, 5 * 60, 10 * 60)  # min 0, max 5, 10 rps/replica, up 5 min, down 10 min


@pytest.mark.parametrize("replicas,rps,expected", [
    pytest.param([_rep()], 10, 0, id="do_not_scale"),
    pytest.param([_rep()], 20, 1, id="scale_up"),
    pytest.param([_rep(), _rep()], 50, 3, id="scale_up_high_load"),
    pytest.param([_rep(), _rep()], 1000, 3, id="scale_up_replicas_limit"),
    pytest.param([_rep(), _rep()], 5, -1, id="scale_down"),
    pytest.param([_rep(ago=60)], 20, 0, id="scale_up_delayed_running"),
    pytest.param([_rep(), _rep(active=False, ago=60)], 20, 0, id="scale_up_delayed_terminated"),
    pytest.param([_rep(), _rep(ago=5 * 60)], 5, 0, id="scale_down_delayed"),
    pytest.param([], 5, 1, id="scale_from_zero_immediately"),
    pytest.param([_rep(active=False, ago=60)], 5, 1, id="scale_from_zero_immediately_terminated"),
    pytest.param([_rep(), _rep()], 0, -2, id="scale_to_zero"),
])
def test_rps_autoscaler(frozen_now, replicas, rps, expected):
    assert _rps().scale(replicas, float(rps)) == expected


# ---- test_docker.py: registry documents, mount targets -------------------------------------------
_MANIFEST = {
    "schemaVersion": 2,
    "mediaType": "application/vnd.oci.image.manifest.v1+json",
    "config": {"mediaType": "application/vnd.oci.image.config.v1+json",
               "digest": "sha256:" + "b5" * 32, "size": 7023},
    "layers": [{"mediaType": "application/vnd.oci.image.layer.v1.tar+gzip", "digest": "sha256:" + "98" * 32,
                "size": 32654}],
    "annotations": {"com.example.key1": "value1"},
}


def _config_object():
    return {
        "created": "2025-03-01T10:00:00Z", "architecture": "amd64", "os": "linux",
        "config": {"User": "alice", "ExposedPorts": {"8080/tcp": {}},
                   "Env": ["PATH=/usr/bin:/bin", "HIP_VISIBLE_DEVICES=0"], "Entrypoint": ["/bin/app"],
                   "Cmd": ["--foreground"], "WorkingDir": "/home/alice", "Labels": {"a": "b"}},
        "rootfs": {"type": "layers", "diff_ids": ["sha256:" + "c6" * 32]},
        "history": [{"created": "2025-03-01T10:00:00Z", "created_by": "/bin/sh -c true"}],
    }


def test_parse_image_manifest():
    from dstack_amd.server.services.docker import parse_image_manifest

    m = parse_image_manifest(_MANIFEST)
    assert m.config.digest == _MANIFEST["config"]["digest"] and len(m.layers) == 1


def test_parse_image_manifest_malformed_is_registry_error():
    from dstack_amd.core.errors import DockerRegistryError
    from dstack_amd.server.services.docker import parse_image_manifest

    with pytest.raises(DockerRegistryError):
        parse_image_manifest({"schemaVersion": 2, "layers": []})


def test_parse_image_config_object():
    from dstack_amd.server.services.docker import parse_image_config_object

    c = parse_image_config_object(_config_object())
    assert c.user == "alice" and c.entrypoint == ["/bin/app"] and c.cmd == ["--foreground"]
    assert "HIP_VISIBLE_DEVICES=0" in c.env


def test_parse_image_config_object_with_config_null():
    from dstack_amd.server.services.docker import parse_image_config_object

    obj = _config_object()
    obj["config"] = None
    c = parse_image_config_object(obj)
    assert c.user is None and c.entrypoint is None and c.env == []


@pytest.mark.parametrize("value,expected", [(None, None), ("", None), ("1000:1000", "1000:1000")])
def test_parse_image_config_object_user_field(value, expected):
    from dstack_amd.server.services.docker import parse_image_config_object

    obj = _config_object()
    obj["config"]["User"] = value
    assert parse_image_config_object(obj).user == expected


def test_parse_image_config_object_user_field_missing():
    from dstack_amd.server.services.docker import parse_image_config_object

    obj = _config_object()
    del obj["config"]["User"]
    assert parse_image_config_object(obj).user is None


@pytest.mark.parametrize("path", ["/valid/path", "/valid-path_with.mixed123", "/valid_path", "/valid.path",
                                  "/valid-path", "/"])
def test_valid_docker_volume_targets(path):
    from dstack_amd.server.services.docker import is_valid_docker_volume_target

    assert is_valid_docker_volume_target(path)


@pytest.mark.parametrize("path", ["invalid/path", "", "relative/path", "./relative/path", "../relative/path",
                                  "/invalid/path/"])
def test_invalid_docker_volume_targets(path):
    from dstack_amd.server.services.docker import is_valid_docker_volume_target

    assert not is_valid_docker_volume_target(path)


def test_run_spec_rejects_volume_inside_workflow(db):
    from tests.test_reconcilers import _submit

    with session_scope() as s, pytest.raises(ServerClientError, match="/workflow"):
        _submit(s, {"type": "task", "commands": ["x"], "volumes": ["/host/data:/workflow/data"]})


# ---- test_fleets.py: SSH hosts belong to one fleet ------------------------------------------------
def _ssh_spec(name, hosts):
    from dstack_amd.core.models.fleets import FleetConfiguration, FleetSpec

    return FleetSpec(configuration=FleetConfiguration.model_validate(
        {"type": "fleet", "name": name, "ssh_config": {"user": "admin", "hosts": hosts,
                                                        "ssh_key": {"public": "ssh-ed25519 AAAA", "private": "k"}}}))


def _project(s, name="main", owner="admin"):
    from dstack_amd.server.services import projects as projects_services
    from dstack_amd.server.services import users as users_services

    p = s.query(ProjectModel).filter_by(name=name).one_or_none()
    if p is not None:
        return p, s.query(UserModel).filter_by(name=owner).one()
    u = s.query(UserModel).filter_by(name=owner).one_or_none() or users_services.create_user(s, owner)
    return projects_services.create_project(s, u, name), u


def _ssh_fleet(s, project, spec):
    from dstack_amd.server.services import pools as pools_services

    f = FleetModel(id=uuid.uuid4(), name=spec.configuration.name, project_id=project.id, status="active",
                   spec=spec.model_dump_json(), created_at=get_current_datetime(),
                   last_processed_at=get_current_datetime())
    s.add(f)
    s.flush()
    pool = pools_services.get_or_create_default_pool(s, project)
    for i, h in enumerate(spec.configuration.ssh_config.hosts):
        host = h if isinstance(h, str) else h.hostname
        rci = RemoteConnectionInfo(host=host, port=22, ssh_user="admin", ssh_keys=[])
        pools_services.create_instance_model(s, project, pool, name=f"{f.name}-{i}", status=InstanceStatus.IDLE,
                                             fleet=f, instance_num=i, backend=BackendType.REMOTE.value,
                                             region="remote", price=0.0, remote_connection_info=rci.model_dump_json())
    return f


def _fleet_plan(s, project, user, spec):
    from dstack_amd.server.services import fleets as fleets_services

    with mock.patch("dstack_amd.server.services.backends.get_project_backends", return_value=[]):
        return fleets_services.get_plan(s, project, user, spec)


def test_ssh_fleet_ok_same_fleet_update(db):
    with session_scope() as s:
        p, u = _project(s)
        _ssh_fleet(s, p, _ssh_spec("my-fleet", ["192.168.100.201"]))
        plan = _fleet_plan(s, p, u, _ssh_spec("my-fleet", ["192.168.100.201", "192.168.100.202"]))
        assert plan.current_resource is not None


def test_ssh_fleet_ok_deleted_instances_ignored(db):
    with session_scope() as s:
        p, u = _project(s)
        f = _ssh_fleet(s, p, _ssh_spec("my-fleet", ["192.168.100.201"]))
        for inst in s.query(InstanceModel).filter_by(fleet_id=f.id):
            inst.deleted = True
        f.deleted = True
        s.flush()
        plan = _fleet_plan(s, p, u, _ssh_spec("my-fleet", ["192.168.100.201", "192.168.100.202"]))
        assert plan.current_resource is None


def test_ssh_fleet_ok_no_common_hosts_with_another_fleet(db):
    with session_scope() as s:
        p, u = _project(s)
        _ssh_fleet(s, p, _ssh_spec("another-fleet", ["192.168.100.201"]))
        plan = _fleet_plan(s, p, u, _ssh_spec("new-fleet", ["192.168.100.202"]))
        assert plan.current_resource is None


def test_ssh_fleet_error_another_fleet_same_project(db):
    with session_scope() as s:
        p, u = _project(s)
        _ssh_fleet(s, p, _ssh_spec("another-fleet", ["192.168.100.201"]))
        with pytest.raises(ServerClientError, match=r"Instances \[192\.168\.100\.201\] are already assigned"):
            _fleet_plan(s, p, u, _ssh_spec("new-fleet", ["192.168.100.201", "192.168.100.202"]))


def test_ssh_fleet_error_another_fleet_another_project(db):
    with session_scope() as s:
        other, _ = _project(s, "another-project", "another-user")
        _ssh_fleet(s, other, _ssh_spec("another-fleet", ["192.168.100.201"]))
        p, u = _project(s, "my-project", "my-user")
        with pytest.raises(ServerClientError, match=r"Instances \[192\.168\.100\.201\] are already assigned"):
            _fleet_plan(s, p, u, _ssh_spec("my-fleet", ["192.168.100.201", "192.168.100.202"]))


def test_ssh_fleet_error_spec_without_name(db):
    # fleets are identified by name: an unnamed spec cannot claim it is the existing fleet
    with session_scope() as s:
        p, u = _project(s)
        _ssh_fleet(s, p, _ssh_spec("autogenerated-fleet-name", ["192.168.100.201"]))
        with pytest.raises(ServerClientError, match=r"Instances \[192\.168\.100\.201\] are already assigned"):
            _fleet_plan(s, p, u, _ssh_spec(None, ["192.168.100.201"]))


def test_ssh_fleet_create_rejects_taken_host(db):
    from dstack_amd.server.services import fleets as fleets_services

    from dstack_amd.utils.common import generate_rsa_key_pair

    private, public = generate_rsa_key_pair()
    spec = _ssh_spec("second", ["10.1.0.5"])
    spec.configuration.ssh_config.ssh_key.private, spec.configuration.ssh_config.ssh_key.public = private, public
    with session_scope() as s:
        p, u = _project(s)
        _ssh_fleet(s, p, _ssh_spec("taken", ["10.1.0.5"]))
        with pytest.raises(ServerClientError, match="already assigned"):
            fleets_services.create_fleet(s, p, u, spec)


# ---- test_pools.py ------------------------------------------------------------------------------
def test_generates_instance_name(db):
    from dstack_amd.server.services import pools as pools_services

    with session_scope() as s:
        p, _ = _project(s)
        pool = pools_services.create_pool(s, p, "test_pool")
        pools_services.create_instance_model(s, p, pool, name="test_instance", status=InstanceStatus.PENDING,
                                             backend=BackendType.REMOTE.value, region="", price=0.0)
        name = pools_services.generate_instance_name(s, p, "test_pool")
        car, _, cdr = name.partition("-")
        assert car and cdr and name != "test_instance"


def test_instance_model_to_instance(db):
    from dstack_amd.core.models.instances import Disk, InstanceType, Resources
    from dstack_amd.server.services import pools as pools_services

    itype = InstanceType(name="instance", resources=Resources(cpus=1, memory_mib=512, spot=False, gpus=[],
                                                              disk=Disk(size_mib=102400)))
    jpd = {"backend": "local", "hostname": "hostname_test", "region": "eu-west", "price": 1.0, "username": "user1",
           "ssh_port": 12345, "dockerized": False, "instance_id": "test_instance",
           "instance_type": itype.model_dump(mode="json")}
    offer = {"backend": "local", "region": "eu-west-1", "price": 1.0, "availability": "available",
             "instance": itype.model_dump(mode="json")}
    with session_scope() as s:
        p, _ = _project(s)
        iid, created = uuid.uuid4(), get_current_datetime()
        im = InstanceModel(id=iid, created_at=created, name="test_instance", instance_num=0,
                           status=InstanceStatus.PENDING.value, unreachable=False, project_id=p.id,
                           job_provisioning_data=json.dumps(jpd), offer=json.dumps(offer), backend="local",
                           region="eu-west-1", price=1.0, total_blocks=1, busy_blocks=0)
        s.add(im)
        s.flush()
        s.refresh(im)
        inst = pools_services.instance_model_to_instance(im)
    assert inst.id == iid and inst.project_name == "main" and inst.backend == BackendType.LOCAL
    assert inst.instance_type == itype and inst.name == "test_instance" and inst.instance_num == 0
    assert inst.hostname == "hostname_test" and inst.status == InstanceStatus.PENDING
    assert inst.region == "eu-west-1" and inst.price == 1.0
    assert (inst.total_blocks, inst.busy_blocks) == (1, 0) and inst.created == created


# ---- test_repos.py ------------------------------------------------------------------------------
_CREDS = {"clone_url": "https://github.com/org/repo.git", "private_key": None, "oauth_token": "user-token"}
_LEGACY = {"clone_url": "https://github.com/org/repo.git", "private_key": None, "oauth_token": "legacy-token"}
_INFO = {"repo_type": "remote", "repo_name": "repo"}


def _remote_repo(s, p, legacy=None):
    r = RepoModel(id=uuid.uuid4(), project_id=p.id, name="gh-repo", type="remote", info=json.dumps(_INFO),
                  creds=json.dumps(legacy) if legacy else None)
    s.add(r)
    s.flush()
    return r


def _head(s, p, u, include_creds=True, repo_id="gh-repo"):
    from dstack_amd.server.services import repos as repos_services

    return repos_services.get_repo_head(s, p, u, repo_id, include_creds)


def test_get_remote_repo_none_if_not_found(db):
    with session_scope() as s:
        p, u = _project(s)
        assert _head(s, p, u) is None


def test_get_remote_repo_without_creds_when_not_requested(db):
    with session_scope() as s:
        p, u = _project(s)
        r = _remote_repo(s, p, legacy=_LEGACY)
        s.add(RepoCredsModel(id=uuid.uuid4(), repo_id=r.id, user_id=u.id, creds=json.dumps(_CREDS)))
        h = _head(s, p, u, include_creds=False)
        assert h.repo_id == "gh-repo" and h.repo_creds is None


def test_get_remote_repo_none_creds_if_no_user_or_legacy_creds(db):
    with session_scope() as s:
        p, u = _project(s)
        _remote_repo(s, p)
        assert _head(s, p, u).repo_creds is None


def test_get_remote_repo_user_creds_if_present(db):
    with session_scope() as s:
        p, u = _project(s)
        r = _remote_repo(s, p, legacy=_LEGACY)
        s.add(RepoCredsModel(id=uuid.uuid4(), repo_id=r.id, user_id=u.id, creds=json.dumps(_CREDS)))
        s.flush()
        assert _head(s, p, u).repo_creds.oauth_token == "user-token"


def test_get_remote_repo_legacy_creds_if_user_creds_not_found(db):
    with session_scope() as s:
        p, u = _project(s)
        r = _remote_repo(s, p, legacy=_LEGACY)
        other = UserModel(id=uuid.uuid4(), name="someone", token="t", token_hash="h", global_role="user")
        s.add(other)
        s.flush()
        s.add(RepoCredsModel(id=uuid.uuid4(), repo_id=r.id, user_id=other.id, creds=json.dumps(_CREDS)))
        s.flush()
        assert _head(s, p, u).repo_creds.oauth_token == "legacy-token"


def _user_creds(s, r, u):
    c = s.query(RepoCredsModel).filter_by(repo_id=r.id, user_id=u.id).one_or_none()
    return json.loads(c.creds) if c else None


def test_init_remote_repo_creates_with_user_creds(db):
    from dstack_amd.server.services import repos as repos_services

    with session_scope() as s:
        p, u = _project(s)
        r = repos_services.init_repo(s, p, u, "gh-repo", _INFO, _CREDS)
        s.flush()
        assert r.type == "remote" and _user_creds(s, r, u) == _CREDS


def test_init_remote_repo_adds_user_creds(db):
    from dstack_amd.server.services import repos as repos_services

    with session_scope() as s:
        p, u = _project(s)
        r = _remote_repo(s, p)
        repos_services.init_repo(s, p, u, "gh-repo", _INFO, _CREDS)
        s.flush()
        assert _user_creds(s, r, u) == _CREDS


def test_init_remote_repo_updates_user_creds(db):
    from dstack_amd.server.services import repos as repos_services

    with session_scope() as s:
        p, u = _project(s)
        r = _remote_repo(s, p)
        repos_services.init_repo(s, p, u, "gh-repo", _INFO, _CREDS)
        new = {**_CREDS, "oauth_token": "rotated"}
        repos_services.init_repo(s, p, u, "gh-repo", _INFO, new)
        s.flush()
        assert _user_creds(s, r, u) == new
        assert s.query(RepoCredsModel).filter_by(repo_id=r.id).count() == 1


def test_init_remote_repo_removes_user_creds(db):
    from dstack_amd.server.services import repos as repos_services

    with session_scope() as s:
        p, u = _project(s)
        r = _remote_repo(s, p)
        repos_services.init_repo(s, p, u, "gh-repo", _INFO, _CREDS)
        s.flush()
        repos_services.init_repo(s, p, u, "gh-repo", _INFO, None)
        s.flush()
        assert _user_creds(s, r, u) is None


# ---- test_runs.py: replica scaling ----------------------------------------------------------------
def _service_run(s, statuses, replicas):
    from dstack_amd.core.models.runs import RunSpec
    from dstack_amd.server.services import jobs as jobs_services
    from tests.test_reconcilers import _submit

    rid = _submit(s, {"type": "service", "commands": ["python -m http.server 8000"], "port": 8000,
                      "replicas": replicas, "scaling": {"metric": "rps", "target": 1}}, name="test-run")
    run = s.get(RunModel, rid)
    for j in list(run.jobs):
        s.delete(j)
    s.flush()
    spec = RunSpec.model_validate_json(run.run_spec)
    for r, st in enumerate(statuses):
        for js in jobs_services.get_jobs_from_run_spec(spec, r, {}):
            j = jobs_services.new_job_model(run, js, submission_num=0)
            j.status = st.value
            s.add(j)
    s.flush()
    s.expire(run)
    return run


def _scale(s, run, diff):
    from dstack_amd.server.services import runs as runs_services

    with mock.patch("dstack_amd.server.services.jobs.stop_runner"):
        runs_services.scale_run_replicas(s, run, diff)
    s.flush()
    s.expire(run)
    return sorted(run.jobs, key=lambda j: (j.submitted_at, j.replica_num, j.submission_num))


def test_scale_no_scale(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.RUNNING], "0..1")
        assert len(_scale(s, run, 0)) == 1


def test_scale_downscale_to_zero(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.RUNNING], "0..1")
        jobs = _scale(s, run, -1)
        assert len(jobs) == 1
        assert jobs[0].status == JobStatus.TERMINATING.value
        assert jobs[0].termination_reason == JobTerminationReason.SCALED_DOWN.value


def test_scale_upscale_new(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.RUNNING], "0..2")
        jobs = _scale(s, run, 1)
        assert len(jobs) == 2
        assert jobs[1].status == JobStatus.SUBMITTED.value and jobs[1].replica_num == 1


def test_scale_upscale_terminated(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.RUNNING, JobStatus.TERMINATED], "0..2")
        jobs = _scale(s, run, 1)
        assert [j.status for j in jobs] == ["running", "terminated", "submitted"]
        assert jobs[2].replica_num == 1 and jobs[2].submission_num == 1  # the old replica, resubmitted


def test_scale_downscale_less_important(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.PROVISIONING, JobStatus.RUNNING], "0..2")
        jobs = _scale(s, run, -1)
        assert [j.status for j in jobs] == ["terminating", "running"]
        assert jobs[0].termination_reason == JobTerminationReason.SCALED_DOWN.value


def test_scale_downscale_greater_replica_num(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.RUNNING, JobStatus.RUNNING], "0..2")
        jobs = _scale(s, run, -1)
        assert [j.status for j in jobs] == ["running", "terminating"]
        assert jobs[1].termination_reason == JobTerminationReason.SCALED_DOWN.value


def test_scale_no_downscale_below_limit(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.RUNNING], "1..2")
        with pytest.raises(ServerClientError, match="minimum"):
            _scale(s, run, -1)


def test_scale_no_upscale_above_limit(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.RUNNING], "0..1")
        with pytest.raises(ServerClientError, match="maximum"):
            _scale(s, run, 1)


def test_scale_upscale_mixed(db):
    with session_scope() as s:
        run = _service_run(s, [JobStatus.TERMINATED], "0..2")
        jobs = _scale(s, run, 2)
        assert [j.status for j in jobs] == ["terminated", "submitted", "submitted"]
        assert [j.replica_num for j in jobs] == [0, 0, 1]


# ---- test_runs.py: can the job's volumes be attached together ---------------------------------------
def _vol(name, region, backend="aws"):
    from dstack_amd.core.models.volumes import VolumeStatus

    conf = {"type": "volume", "name": name, "backend": backend, "region": region, "size": 100}
    return VolumeModel(id=uuid.uuid4(), name=name, status=VolumeStatus.ACTIVE.value,
                       configuration=json.dumps(conf))


def test_can_attach_volumes_with_alternatives_per_region():
    from dstack_amd.server.services.jobs.volumes import check_can_attach_job_volumes

    check_can_attach_job_volumes([[_vol("vol11", "eu-west-1"), _vol("vol12", "eu-west-2")],
                                  [_vol("vol21", "eu-west-1"), _vol("vol22", "eu-west-2")]])


def test_cannot_attach_mount_points_in_different_regions():
    from dstack_amd.server.services.jobs.volumes import check_can_attach_job_volumes

    with pytest.raises(ServerClientError):
        check_can_attach_job_volumes([[_vol("vol1", "eu-west-1")], [_vol("vol2", "eu-west-2")]])


def test_cannot_attach_same_volume_at_different_mount_points():
    from dstack_amd.server.services.jobs.volumes import check_can_attach_job_volumes

    v = _vol("vol1", "eu-west-1")
    with pytest.raises(ServerClientError, match="same volume"):
        check_can_attach_job_volumes([[v], [v]])


# ---- jobs/configurators/test_base.py: interpolate_job_volumes -------------------------------------
@pytest.mark.parametrize("run_volumes,job_num,expected", [
    pytest.param([VolumeMountPoint(name="volume", path="/volume")], 0,
                 [VolumeMountPoint(name=["volume"], path="/volume")], id="no_interpolation"),
    pytest.param([InstanceMountPoint(instance_path="/volume", path="/volume")], 0,
                 [InstanceMountPoint(instance_path="/volume", path="/volume")], id="instance_mount"),
    pytest.param([VolumeMountPoint(name="job${{dstack.job_num}}-rank${{dstack.node_rank}}", path="/volume")], 2,
                 [VolumeMountPoint(name=["job2-rank2"], path="/volume")], id="job_num_and_node_rank"),
])
def test_interpolates_job_volumes(run_volumes, job_num, expected):
    from dstack_amd.server.services.jobs.configurators import interpolate_job_volumes

    assert interpolate_job_volumes(run_volumes, job_num) == expected


@pytest.mark.parametrize("name", ["${{}", "${{ unknown.namespace }}", "${{ dstack.var }}"],
                         ids=["invalid_syntax", "unknown_namespace", "unknown_var"])
def test_interpolate_job_volumes_errors_are_client_errors(name):
    from dstack_amd.server.services.jobs.configurators import interpolate_job_volumes

    with pytest.raises(ServerClientError):
        interpolate_job_volumes([VolumeMountPoint(name=name, path="/volume")], 0)
