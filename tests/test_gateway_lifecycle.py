"""Gateway lifecycle on the server: the cloud VM is terminated on delete (and the gateway kept when
that fails), gateways are reconnected / updated blue-green / re-configured at server start, and the
versioned gateway package + update.sh switch slots and roll back (reference:
``S/services/gateways/__init__.py:226-255,356-430``, ``gateway/`` packaging)."""

import json
import os
import subprocess
import tarfile
import urllib.parse
import uuid
from unittest import mock

import httpx
import pytest

from dstack_amd.server.db import session_scope
from dstack_amd.server.models import BackendModel, GatewayComputeModel, GatewayModel, ProjectModel
from dstack_amd.utils.common import get_current_datetime


def _aws_gateway(s, name="gw", instance_id="i-gw1"):
    project = s.query(ProjectModel).filter_by(name="main").one()
    be = s.query(BackendModel).filter_by(project_id=project.id, type="aws").one_or_none()
    if be is None:
        be = BackendModel(id=uuid.uuid4(), project_id=project.id, type="aws", config="{}",
                          auth=json.dumps({"access_key": "AK", "secret_key": "SK"}))
        s.add(be)
        s.flush()
    comp = GatewayComputeModel(id=uuid.uuid4(), instance_id=instance_id, ip_address="3.3.3.3", region="us-east-1",
                               backend_id=be.id, ssh_private_key="k", ssh_public_key="ssh-rsa AAA gw",
                               backend_data=None)
    s.add(comp)
    s.flush()
    g = GatewayModel(id=uuid.uuid4(), name=name, region="us-east-1", project_id=project.id, backend_id=be.id,
                     configuration=json.dumps({"type": "gateway", "name": name, "backend": "aws",
                                               "region": "us-east-1", "domain": "example.com"}),
                     status="running", wildcard_domain="example.com", gateway_compute_id=comp.id,
                     created_at=get_current_datetime(), last_processed_at=get_current_datetime())
    s.add(g)
    s.flush()
    return g.id, comp.id


def _aws(handler):
    from dstack_amd.core.backends.clouds.aws import AWSCompute

    return AWSCompute({}, {"access_key": "AK", "secret_key": "SK"}, httpx.Client(transport=httpx.MockTransport(handler)))


def _xml(body):
    return f'<Response xmlns="http://ec2.amazonaws.com/doc/2016-11-15/">{body}</Response>'


def test_delete_cloud_gateway_terminates_its_vm(client):
    from dstack_amd.server.services import backends as backends_services

    calls = []

    def handler(req):
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        calls.append((form["Action"], form.get("InstanceId.1")))
        return httpx.Response(200, text=_xml(""))

    with session_scope() as s:
        gid, cid = _aws_gateway(s)
    with mock.patch.object(backends_services, "get_project_backend", return_value=_aws(handler)):
        r = client.post("/api/project/main/gateways/delete", json={"names": ["gw"]})
    assert r.status_code == 200, r.text
    assert calls == [("TerminateInstances", "i-gw1")]
    with session_scope() as s:
        assert s.get(GatewayModel, gid) is None
        comp = s.get(GatewayComputeModel, cid)
        assert comp.deleted and not comp.active


def test_gateway_kept_when_its_vm_cannot_be_terminated(client):
    from dstack_amd.server.services import backends as backends_services

    def handler(req):
        return httpx.Response(500, text=_xml("<Errors><Error><Code>InternalError</Code><Message>boom</Message>"
                                             "</Error></Errors>"))

    with session_scope() as s:
        gid, cid = _aws_gateway(s)
        _aws_gateway(s, name="gw-ok", instance_id="i-gw2")
    ok_calls = []

    def ok_handler(req):
        ok_calls.append(dict(urllib.parse.parse_qsl(req.content.decode())).get("InstanceId.1"))
        return httpx.Response(200, text=_xml(""))

    with mock.patch.object(backends_services, "get_project_backend", side_effect=lambda *a: _aws(handler)), \
            mock.patch("time.sleep"):
        r = client.post("/api/project/main/gateways/delete", json={"names": ["gw"]})
    assert r.status_code == 400 and "retry" in r.text
    with session_scope() as s:
        g = s.get(GatewayModel, gid)
        assert g is not None and g.gateway_compute.active and not g.gateway_compute.deleted
    # a later delete that succeeds removes it
    with mock.patch.object(backends_services, "get_project_backend", return_value=_aws(ok_handler)):
        assert client.post("/api/project/main/gateways/delete", json={"names": ["gw", "gw-ok"]}).status_code == 200
    assert sorted(ok_calls) == ["i-gw1", "i-gw2"]


def test_init_gateways_updates_outdated_app_once_and_configures(db):
    from dstack_amd.server.services import gateways as gw_services

    from datetime import timedelta

    with session_scope() as s:
        gid, cid = _aws_gateway(s)
        # installed an hour ago (a gateway created or updated within the last minute is not updated)
        s.get(GatewayComputeModel, cid).app_updated_at = get_current_datetime() - timedelta(hours=1)
    sent = []

    def fake_call(g, method, path, body=None):
        sent.append((method, path, body))
        if path == "/api/healthcheck":
            return {"service": "dstack-gateway", "version": "0.0.1"}
        return {}

    with mock.patch.object(gw_services, "_call", side_effect=fake_call), \
            mock.patch.object(gw_services, "update_gateway_app", return_value=True) as upd:
        assert gw_services.init_gateways(skip_update=False) == {"gw": "updated"}
        upd.assert_called_once()
        assert ("POST", "/api/config") in [(m, p) for m, p, _ in sent]
        # updated less than a minute ago: the next server start does not update again
        assert gw_services.init_gateways(skip_update=False) == {"gw": "connected"}
        assert upd.call_count == 1
    with mock.patch.object(gw_services, "_call", side_effect=httpx.ConnectError("down")):
        assert gw_services.init_gateways() == {"gw": "unreachable"}


def test_init_gateways_skip_update(db):
    from dstack_amd.server.services import gateways as gw_services

    with session_scope() as s:
        _aws_gateway(s)
    with mock.patch.object(gw_services, "_call", return_value={"version": "0.0.1"}), \
            mock.patch.object(gw_services, "update_gateway_app") as upd:
        assert gw_services.init_gateways(skip_update=True) == {"gw": "connected"}
    upd.assert_not_called()


def test_update_gateway_app_pushes_script_and_runs_blue_green(db):
    from dstack_amd.proxy.gateway import packaging
    from dstack_amd.server.services import gateways as gw_services

    with session_scope() as s:
        gid, cid = _aws_gateway(s)
    runs = []

    class Pool:
        def run(self, target, key, command, timeout=600, input=None):
            runs.append((target.hostname, command, input))
            out = b"Update successfully completed\n" if "_update.sh" in command else b""
            return subprocess.CompletedProcess([], 0, out, b"")

    with mock.patch("dstack_amd.core.services.ssh.tunnel.get_tunnel_pool", return_value=Pool()), session_scope() as s:
        assert gw_services.update_gateway_app(s.get(GatewayComputeModel, cid), version="9.9.9", url="http://pkg/x")
    assert runs[0][1].endswith("cat > dstack/update.sh") and runs[0][2] == packaging.UPDATE_SH.encode()
    assert "sh dstack/_update.sh 'http://pkg/x' '9.9.9'" in runs[1][1] and runs[1][0] == "3.3.3.3"


def test_local_gateway_relaunched_with_its_services_on_server_start(client, tmp_path, monkeypatch):
    from dstack_amd.server.services import gateways as gw_services

    r = client.post("/api/project/main/gateways/create", json={"configuration": {
        "type": "gateway", "name": "lgw", "backend": "local", "region": "local", "domain": "local.test"}})
    assert r.status_code == 200, r.text
    with session_scope() as s:
        g = s.query(GatewayModel).filter_by(name="lgw").one()
        gw_services.provision_gateway(s, g)
        assert g.status == "running"
        gid = g.id
    try:
        with session_scope() as s:
            g = s.get(GatewayModel, gid)
            gw_services._call(g, "POST", "/api/registry/main/services/register",
                              {"run_name": "svc", "domain": "svc.local.test", "https": False, "auth": False})
        gw_services.LocalGatewayProcess.stop_all()  # the server stops: its local gateway goes too
        assert gw_services.init_gateways() == {"lgw": "restarted"}
        with session_scope() as s:
            g = s.get(GatewayModel, gid)
            health = gw_services._call(g, "GET", "/api/healthcheck")
        assert health["services"] == 1 and health["version"]
        assert gw_services.init_gateways() == {"lgw": "running"}
    finally:
        gw_services.LocalGatewayProcess.stop_all()


# ---- packaging + update.sh ---------------------------------------------------------------------
def test_gateway_package_is_versioned_and_deterministic(tmp_path):
    from dstack_amd.proxy.gateway import packaging

    a = packaging.build_package(str(tmp_path / "a"), version="1.2.3")
    b = packaging.build_package(str(tmp_path / "b"), version="1.2.3")
    assert os.path.basename(a) == "dstack_amd-gateway-1.2.3.tar.gz"
    assert open(a, "rb").read() == open(b, "rb").read()
    with tarfile.open(a) as t:
        names = set(t.getnames())
        assert t.extractfile("VERSION").read() == b"1.2.3"
    assert {"dstack_amd/__init__.py", "dstack_amd/proxy/gateway/app.py", "dstack_amd/proxy/gateway/main.py",
            "requirements.txt"} <= names
    assert not any("__pycache__" in n for n in names)


@pytest.fixture
def gw_host(tmp_path):
    """A fake gateway host: $ROOT with the slots, a fake ``curl`` that answers the healthcheck with
    the VERSION of the slot ``current`` points at (or a stale version when BROKEN exists)."""
    root = tmp_path / "dstack"
    root.mkdir()
    bindir = tmp_path / "bin"
    bindir.mkdir()
    curl = bindir / "curl"
    curl.write_text("#!/bin/sh\n"
                    "if [ -f \"$DSTACK_GATEWAY_ROOT/BROKEN\" ]; then echo '{\"version\":\"0.0.0\"}'; exit 0; fi\n"
                    "printf '{\"service\":\"dstack-gateway\",\"version\":\"%s\"}' "
                    "\"$(cat \"$DSTACK_GATEWAY_ROOT/current/src/VERSION\")\"\n")
    curl.chmod(0o755)
    script = tmp_path / "update.sh"
    from dstack_amd.proxy.gateway import packaging

    script.write_text(packaging.UPDATE_SH)
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", DSTACK_GATEWAY_ROOT=str(root),
               DSTACK_GATEWAY_RESTART="true", DSTACK_GATEWAY_HEALTH_TRIES="2", DSTACK_GATEWAY_HEALTH_SLEEP="0",
               DSTACK_GATEWAY_SKIP_PIP="1")

    def run(pkg, version):
        return subprocess.run(["sh", str(script), pkg, version], env=env, capture_output=True, text=True, timeout=60)

    return root, run


def test_update_sh_installs_switches_and_rolls_back(tmp_path, gw_host):
    from dstack_amd.proxy.gateway import packaging

    root, run = gw_host
    p1 = packaging.build_package(str(tmp_path / "p"), version="1.0.0")
    r = run(p1, "1.0.0")
    assert r.returncode == 0 and "Update successfully completed" in r.stdout, r.stdout + r.stderr
    assert os.readlink(root / "current").endswith("blue")
    assert (root / "current" / "src" / "dstack_amd" / "proxy" / "gateway" / "app.py").exists()
    p2 = packaging.build_package(str(tmp_path / "p"), version="2.0.0")
    r = run(p2, "2.0.0")
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.readlink(root / "current").endswith("green")
    # wrong version in the package: refused before anything is switched
    r = run(p2, "3.0.0")
    assert r.returncode == 1 and "!=" in r.stdout
    assert os.readlink(root / "current").endswith("green")
    # the new app never becomes healthy: switched back to the previous slot
    (root / "BROKEN").write_text("")
    p3 = packaging.build_package(str(tmp_path / "p"), version="3.0.0")
    r = run(p3, "3.0.0")
    assert r.returncode == 1 and "rolling back" in r.stdout and "successfully" not in r.stdout
    assert os.readlink(root / "current").endswith("green")
    assert (root / "current" / "src" / "VERSION").read_text() == "2.0.0"


def test_gateway_cloud_init_installs_versioned_package():
    from dstack_amd.core.backends.clouds.gateway_boot import gateway_cloud_init
    from dstack_amd.core.models.backends import BackendType
    from dstack_amd.core.models.gateways import GatewayComputeConfiguration

    ci = gateway_cloud_init(GatewayComputeConfiguration(project_name="main", instance_name="gw", backend=BackendType.AWS,
                                                        region="us-east-1", public_ip=True,
                                                        ssh_key_pub="ssh-rsa AAA x"))
    assert "dstack_amd-gateway-" in ci and "update.sh" in ci and "base64 -d > /etc/systemd/system/dstack-gateway" in ci


def test_private_gateway_only_where_supported(client):
    """``public_ip: false`` is refused up front on backends without private gateways."""
    body = {"configuration": {"type": "gateway", "name": "gw-priv", "backend": "gcp", "region": "us-central1",
                              "domain": "gw.example.com", "public_ip": False}}
    r = client.post("/api/project/main/gateways/create", json=body)
    assert r.status_code == 400 and "without a public IP" in r.text, r.text
