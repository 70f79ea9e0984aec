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


def test_oci_backend_not_created_if_regions_not_subscribed(client, fake_oci):
    r = client.post("/api/project/main/backends/create", json=_oci_body(["us-chicago-1", "eu-frankfurt-1"]))
    assert r.status_code == 400 and "eu-frankfurt-1" in r.text and "not subscribed" in r.text, r.text
    assert {region for _, region, _, _ in fake_oci.calls} == {"us-chicago-1"}  # the key's home region answers
    assert not [c for c in fake_oci.calls if c[0] == "POST"]  # nothing created for a refused config
    assert client.post("/api/project/main/backends/create", json=_oci_body(["us-chicago-1"])).status_code == 200


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


class _FakeOCI:
    """In-memory OCI control plane for the paths the backend uses (identity + core services)."""

    def __init__(self):
        self.calls = []
        self.objs = {}  # kind -> list of dicts
        self.n = 0

    def _store(self, kind, region):
        key = kind if kind == "compartments" else f"{region}/{kind}"
        return self.objs.setdefault(key, [])

    def _new(self, kind, body, region, state="PROVISIONING"):
        self.n += 1
        obj = {**body, "id": f"ocid1.{kind}.{self.n}", "lifecycleState": state}
        if kind == "vcns":
            obj["defaultRouteTableId"] = f"ocid1.rt.{self.n}"
            obj["defaultSecurityListId"] = f"ocid1.sl.{self.n}"
            self._store("routeTables", region).append({"id": obj["defaultRouteTableId"], "routeRules": [],
                                                       "lifecycleState": "AVAILABLE"})
            self._store("securityLists", region).append({
                "id": obj["defaultSecurityListId"], "lifecycleState": "AVAILABLE",
                # OCI's default list: SSH from anywhere, as the API returns it (ids, timestamps, defaults)
                "ingressSecurityRules": [{"protocol": "6", "source": "0.0.0.0/0", "sourceType": "CIDR_BLOCK",
                                          "isStateless": False, "id": "r1", "timeCreated": "2024-01-01T00:00:00Z",
                                          "tcpOptions": {"destinationPortRange": {"min": 22, "max": 22},
                                                         "sourcePortRange": None}},
                                         {"protocol": "6", "source": "192.168.0.0/16", "isStateless": False,
                                          "tcpOptions": {"destinationPortRange": {"min": 9000, "max": 9000}}}],
                "egressSecurityRules": []})
        self._store(kind, region).append(obj)
        return obj

    def __call__(self, comp, method, region, path, body=None, host=None):
        from urllib.parse import parse_qsl, urlsplit

        self.calls.append((method, region, path.split("?")[0], body))
        u = urlsplit(path)
        parts = u.path.split("/")[2:]  # drop "" and the API version
        q = dict(parse_qsl(u.query))
        req = httpx.Request(method, f"https://{host or 'iaas'}{path}")

        def ok(obj, status=200):
            return httpx.Response(status, json=obj, request=req)

        kind = parts[0]
        if kind == "users":
            return ok({"id": parts[1]})
        if kind == "tenancies":
            return ok([{"regionName": "us-chicago-1"}, {"regionName": "us-ashburn-1"}])
        if method == "GET" and len(parts) == 1:
            items = self._store(kind, region)
            name = q.get("displayName") or q.get("name")
            for o in items:  # every object becomes AVAILABLE after one look
                o["lifecycleState"] = "ACTIVE" if kind == "compartments" else "AVAILABLE"
            return ok([o for o in items if name is None or o.get("displayName", o.get("name")) == name])
        if method == "GET":
            o = next(o for o in self._store(kind, region) if o["id"] == parts[1])
            o["lifecycleState"] = "ACTIVE" if kind == "compartments" else "AVAILABLE"
            return ok(o)
        if method == "POST" and len(parts) == 1:
            return ok(self._new(kind, body, region))
        if method == "PUT":
            o = next(o for o in self._store(kind, region) if o["id"] == parts[1])
            o.update(body)
            return ok(o)
        raise AssertionError(f"unexpected OCI call {method} {path}")


@pytest.fixture
def fake_oci(monkeypatch):
    from dstack_amd.core.backends.clouds.hyperscalers import OCICompute

    monkeypatch.delenv("DSTACK_SKIP_BACKEND_VALIDATION", raising=False)
    monkeypatch.setattr(OCICompute, "WAIT_S", 5.0)
    monkeypatch.setattr(OCICompute, "WAIT_POLL_S", 0.0)
    fake = _FakeOCI()
    monkeypatch.setattr(OCICompute, "_signed", lambda self, *a, **k: fake(self, *a, **k))
    return fake


def _oci_body(regions):
    from dstack_amd.utils.common import generate_rsa_key_pair

    body = json.loads(json.dumps(VALID["oci"]))
    body["creds"]["key_content"] = generate_rsa_key_pair()[0]
    body["regions"] = regions
    return body


def test_oci_backend_creation_bootstraps_the_network(client, fake_oci):
    """(verdict: OCI network bootstrap; reference ``oci/resources.py:427-690``) creating the backend
    creates the compartment, and per region the VCN, internet gateway, default route, security
    rules and a subnet; their ids are stored in the backend's config."""
    r = client.post("/api/project/main/backends/create", json=_oci_body(["us-chicago-1"]))
    assert r.status_code == 200, r.text
    posts = [p for m, _, p, _ in fake_oci.calls if m == "POST"]
    assert posts == ["/20160918/compartments", "/20160918/vcns", "/20160918/internetGateways", "/20160918/subnets"]
    objs = {k.split("/")[-1]: v for k, v in fake_oci.objs.items()}  # one region here
    rt = objs["routeTables"][0]["routeRules"]
    assert rt == [{"destination": "0.0.0.0/0", "destinationType": "CIDR_BLOCK",
                   "networkEntityId": objs["internetGateways"][0]["id"]}]
    ingress = objs["securityLists"][0]["ingressSecurityRules"]
    from dstack_amd.core.backends.clouds.hyperscalers import SecurityRule

    rules = [SecurityRule.from_api(x, "INGRESS") for x in ingress]
    assert SecurityRule("INGRESS", "all", "10.0.0.0/16") in rules  # node-to-node (RCCL) traffic
    assert SecurityRule("INGRESS", "6", "192.168.0.0/16", ports=(9000, 9000)) in rules  # the user's rule is kept
    assert any(x.get("tcpOptions", {}).get("destinationPortRange") == {"min": 22, "max": 22} for x in ingress)
    info = client.post("/api/project/main/backends/oci/config_info").json()
    assert info["compartment_id"] == fake_oci.objs["compartments"][0]["id"]
    assert info["subnet_ids"] == {"us-chicago-1": objs["subnets"][0]["id"]}


def test_oci_network_bootstrap_is_idempotent_and_lazy_for_new_regions(fake_oci):
    from dstack_amd.core.backends.clouds.hyperscalers import OCICompute

    auth = {"user": "u", "tenancy": "t", "fingerprint": "f", "region": "us-chicago-1", "key_content": "k"}
    comp = OCICompute({"regions": ["us-chicago-1"]}, auth, None)
    first = comp.ensure_network("us-chicago-1")
    n_writes = sum(1 for m, *_ in fake_oci.calls if m in ("POST", "PUT"))
    again = OCICompute({"regions": ["us-chicago-1"]}, auth, None).ensure_network("us-chicago-1")
    # nothing created or rewritten the second time (the security rules read back compare equal)
    assert again == first and sum(1 for m, *_ in fake_oci.calls if m in ("POST", "PUT")) == n_writes
    # a region without a recorded subnet gets its own VCN + subnet at launch
    assert comp.ensure_network("us-ashburn-1") != first
    assert set(comp.config["subnet_ids"]) == {"us-chicago-1", "us-ashburn-1"}
