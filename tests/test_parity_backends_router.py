"""Backends router, case by case against the reference's ``routers/test_backends.py`` (mapping:
``docs/reference/test-parity.md``): form values per cloud with and without credentials (the cloud's
verdict is stubbed -- there is no network), deletion refused while a backend still owns instances or
volumes, OCI regions the tenancy has not subscribed, and config info / YAML round trips.  Creation
per cloud and the secret split are in ``test_backends_api.py``; the 403 / 40x cases in
``test_api_access_matrix.py``."""

from __future__ import annotations

import json
import uuid

import httpx
import pytest
import yaml

from dstack_amd.core.errors import BackendAuthError
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import InstanceModel, ProjectModel, VolumeModel
from dstack_amd.utils.common import get_current_datetime
from tests.test_backends_api import VALID

CLOUDS = ["aws", "azure", "gcp", "lambda", "oci"]


@pytest.fixture
def cloud_verdict(monkeypatch):
    """Credentials check answered locally: ``bad`` anywhere in the creds -> rejected."""
    from dstack_amd.core.backends import clouds

    monkeypatch.delenv("DSTACK_SKIP_BACKEND_VALIDATION", raising=False)
    seen = []

    class _Fake:
        def __init__(self, cfg, auth, http):
            self.auth = auth

        def check_credentials(self):
            seen.append(dict(self.auth))
            if "bad" in json.dumps(self.auth):
                raise BackendAuthError("rejected by the cloud")

    monkeypatch.setattr(clouds, "compute_class", lambda bt: _Fake)
    return seen


@pytest.mark.parametrize("btype", CLOUDS)
def test_config_values_initial_without_creds(client, cloud_verdict, btype):
    r = client.post("/api/backends/config_values", json={"type": btype})
    assert r.status_code == 200, r.text
    out = r.json()
    assert out["type"] == btype and out["regions"]["values"], out
    assert out["default_creds"] == (btype != "lambda")
    assert cloud_verdict == []  # nothing to check yet


def _with_creds(btype, bad):
    body = json.loads(json.dumps(VALID[btype]))
    key = next(k for k, v in body["creds"].items() if k != "type" and isinstance(v, str))
    body["creds"][key] = "bad" if bad else body["creds"][key]
    return body


@pytest.mark.parametrize("btype", CLOUDS)
def test_config_values_invalid_credentials(client, cloud_verdict, btype):
    r = client.post("/api/backends/config_values", json=_with_creds(btype, bad=True))
    assert r.status_code == 400, r.text
    assert r.json()["detail"][0]["code"] == "invalid_credentials"
    assert len(cloud_verdict) == 1


@pytest.mark.parametrize("btype", CLOUDS)
def test_config_values_on_valid_credentials(client, cloud_verdict, btype):
    r = client.post("/api/backends/config_values", json=_with_creds(btype, bad=False))
    assert r.status_code == 200, r.text
    assert r.json()["regions"]["values"] and len(cloud_verdict) == 1


def test_oci_backend_not_created_if_regions_not_subscribed(client, monkeypatch):
    from dstack_amd.core.backends.clouds.hyperscalers import OCICompute
    from dstack_amd.utils.common import generate_rsa_key_pair

    monkeypatch.delenv("DSTACK_SKIP_BACKEND_VALIDATION", raising=False)
    asked = []

    def signed(self, method, region, path, body=None, host=None):
        asked.append((region, path))
        req = httpx.Request(method, f"https://{host}{path}")
        if path.endswith("/regionSubscriptions"):
            return httpx.Response(200, json=[{"regionName": "us-chicago-1"}, {"regionName": "us-ashburn-1"}],
                                  request=req)
        return httpx.Response(200, json={"id": "ocid1.user"}, request=req)

    monkeypatch.setattr(OCICompute, "_signed", signed)
    private, _ = generate_rsa_key_pair()
    body = json.loads(json.dumps(VALID["oci"]))
    body["creds"]["key_content"] = private
    body["regions"] = ["us-chicago-1", "eu-frankfurt-1"]
    r = client.post("/api/project/main/backends/create", json=body)
    assert r.status_code == 400 and "eu-frankfurt-1" in r.text and "not subscribed" in r.text, r.text
    assert all(region == "us-chicago-1" for region, _ in asked)  # the key's home region answers
    body["regions"] = ["us-chicago-1"]
    assert client.post("/api/project/main/backends/create", json=body).status_code == 200


def _project_id():
    with session_scope() as s:
        return s.query(ProjectModel).filter_by(name="main").one().id


def test_delete_backend_with_active_instances_400(client):
    assert client.post("/api/project/main/backends/create", json=VALID["aws"]).status_code == 200
    with session_scope() as s:
        inst = InstanceModel(id=uuid.uuid4(), name="i1", instance_num=0, project_id=_project_id(), backend="aws",
                             region="us-east-1", price=1.0, status="idle", unreachable=False,
                             created_at=get_current_datetime(), last_processed_at=get_current_datetime())
        s.add(inst)
        iid = inst.id
    r = client.post("/api/project/main/backends/delete", json={"backends_names": ["aws"]})
    assert r.status_code == 400 and "active instances" in r.text
    with session_scope() as s:
        s.get(InstanceModel, iid).status = "terminated"
    assert client.post("/api/project/main/backends/delete", json={"backends_names": ["aws"]}).status_code == 200
    assert client.post("/api/project/main/backends/aws/config_info").status_code == 400


def test_delete_backend_with_active_volumes_400(client):
    from dstack_amd.server.models import UserModel

    assert client.post("/api/project/main/backends/create", json=VALID["aws"]).status_code == 200
    with session_scope() as s:
        admin = s.query(UserModel).filter_by(name="admin").one()
        v = VolumeModel(id=uuid.uuid4(), name="v1", user_id=admin.id, project_id=_project_id(), status="active",
                        configuration=json.dumps({"type": "volume", "name": "v1", "backend": "aws",
                                                  "region": "us-east-1", "size": 100}))
        s.add(v)
        vid = v.id
    r = client.post("/api/project/main/backends/delete", json={"backends_names": ["aws"]})
    assert r.status_code == 400 and "active volumes" in r.text
    with session_scope() as s:
        s.get(VolumeModel, vid).deleted = True
    assert client.post("/api/project/main/backends/delete", json={"backends_names": ["aws"]}).status_code == 200


def test_config_info_returns_settings_without_secrets(client):
    client.post("/api/project/main/backends/create", json=VALID["aws"])
    info = client.post("/api/project/main/backends/aws/config_info").json()
    assert info == {"type": "aws", "regions": ["us-east-1"]} or (info["type"] == "aws" and "creds" not in info)


def test_yaml_create_update_and_get(client):
    y = yaml.safe_dump(VALID["oci"])
    assert client.post("/api/project/main/backends/create_yaml", json={"config_yaml": y}).status_code == 200
    upd = {**VALID["oci"], "regions": ["us-ashburn-1"]}
    r = client.post("/api/project/main/backends/update_yaml", json={"config_yaml": yaml.safe_dump(upd)})
    assert r.status_code == 200, r.text
    got = yaml.safe_load(client.post("/api/project/main/backends/oci/get_yaml").json()["config_yaml"])
    assert got["type"] == "oci" and got["regions"] == ["us-ashburn-1"] and "creds" not in got
