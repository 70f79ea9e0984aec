"""Cloud backends against mock HTTP transports (reference analogue: ``src/tests/_internal/core/
backends/*``): request shapes, auth/signing, the create -> poll -> terminate flow, capacity errors."""

import base64
import os
import json
import re
import subprocess
import urllib.parse

import httpx
import pytest

from dstack_amd.core.backends.clouds import compute_class
from dstack_amd.core.backends.clouds.common import sigv4_headers
from dstack_amd.core.errors import NoCapacityError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import InstanceConfiguration, SSHKey
from dstack_amd.core.models.runs import Requirements
from dstack_amd.core.models.resources import ResourcesSpec

CFG = InstanceConfiguration(project_name="main", instance_name="run-0-0", user="admin",
                            ssh_keys=[SSHKey(public="ssh-ed25519 AAAA test@dstack")])


def _client(handler):
    return httpx.Client(transport=httpx.MockTransport(handler))


def _offer(compute, gpu="MI300X"):
    req = Requirements(resources=ResourcesSpec.model_validate({"gpu": gpu}))
    offers = compute.get_offers(req)
    assert offers, f"no {gpu} offers for {compute.TYPE}"
    return offers[0]


# ---- AWS --------------------------------------------------------------------------------------
def test_sigv4_known_vector():
    """AWS documentation's GetSessionToken-style vector shape: deterministic for fixed inputs."""
    import datetime as dt

    h = sigv4_headers("GET", "https://iam.amazonaws.com/?Action=ListUsers&Version=2010-05-08", "us-east-1", "iam",
                      "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY",
                      now=dt.datetime(2015, 8, 30, 12, 36, 0, tzinfo=dt.timezone.utc))
    assert h["x-amz-date"] == "20150830T123600Z"
    assert h["Authorization"].startswith("AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/20150830/us-east-1/iam/aws4_request")
    again = sigv4_headers("GET", "https://iam.amazonaws.com/?Action=ListUsers&Version=2010-05-08", "us-east-1", "iam",
                          "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY",
                          now=dt.datetime(2015, 8, 30, 12, 36, 0, tzinfo=dt.timezone.utc))
    assert h == again


def _xml(body):
    return f'<Response xmlns="http://ec2.amazonaws.com/doc/2016-11-15/">{body}</Response>'


def test_aws_run_describe_terminate():
    calls = []

    def handler(req: httpx.Request):
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        calls.append(form["Action"])
        assert req.headers["authorization"].startswith("AWS4-HMAC-SHA256 Credential=AK/")
        a = form["Action"]
        if a == "DescribeImages":
            return httpx.Response(200, text=_xml("<imagesSet><item><imageId>ami-1</imageId><creationDate>2024"
                                                 "</creationDate></item></imagesSet>"))
        if a == "DescribeSecurityGroups":
            return httpx.Response(200, text=_xml("<securityGroupInfo><item><groupId>sg-1</groupId></item>"
                                                 "</securityGroupInfo>"))
        if a == "RunInstances":
            assert form["InstanceType"] == "p5.48xlarge" and form["ImageId"] == "ami-1"
            ud = base64.b64decode(form["UserData"]).decode()
            assert ud.startswith("#cloud-config") and "dstack-shim" in ud
            return httpx.Response(200, text=_xml("<instancesSet><item><instanceId>i-123</instanceId></item>"
                                                 "</instancesSet>"))
        if a == "DescribeInstances":
            return httpx.Response(200, text=_xml("<reservationSet><item><instancesSet><item><instanceId>i-123"
                                                 "</instanceId><instanceState><name>running</name></instanceState>"
                                                 "<ipAddress>3.3.3.3</ipAddress><privateIpAddress>10.0.0.3"
                                                 "</privateIpAddress></item></instancesSet></item></reservationSet>"))
        if a == "TerminateInstances":
            return httpx.Response(200, text=_xml(""))
        return httpx.Response(400, text=_xml("<Errors><Error><Code>Bad</Code></Error></Errors>"))

    c = compute_class(BackendType.AWS)({}, {"access_key": "AK", "secret_key": "SK"}, _client(handler))
    offer = _offer(c, "H100:8")
    jpd = c.create_instance(offer, CFG)
    assert jpd.instance_id == "i-123" and jpd.hostname is None
    c.update_provisioning_data(jpd)
    assert jpd.hostname == "3.3.3.3" and jpd.internal_ip == "10.0.0.3"
    c.terminate_instance(jpd.instance_id, jpd.region, jpd.backend_data)
    assert calls[-1] == "TerminateInstances"


def test_aws_capacity_error():
    def handler(req):
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        if form["Action"] == "RunInstances":
            return httpx.Response(500, text=_xml("<Errors><Error><Code>InsufficientInstanceCapacity</Code>"
                                                 "<Message>none</Message></Error></Errors>"))
        if form["Action"] == "DescribeImages":
            return httpx.Response(200, text=_xml("<imagesSet><item><imageId>ami-1</imageId></item></imagesSet>"))
        return httpx.Response(200, text=_xml("<securityGroupInfo><item><groupId>sg</groupId></item>"
                                             "</securityGroupInfo>"))

    c = compute_class(BackendType.AWS)({}, {"access_key": "AK", "secret_key": "SK"}, _client(handler))
    with pytest.raises(NoCapacityError):
        c.create_instance(_offer(c, "H100:8"), CFG)


# ---- Vultr (MI355X bare metal) -----------------------------------------------------------------
def test_vultr_mi355x_bare_metal():
    """Bare-metal MI355X node: launched into the region's dstack VPC (created once, reused), the
    host firewall opened to the VPC subnet, and the node's VPC address reported as its internal IP
    (what cluster peers use for RCCL / torchrun)."""
    state = {"status": "pending"}
    vpcs, posts = [], []

    def handler(req):
        assert req.headers["authorization"] == "Bearer vk"
        if req.url.path == "/v2/vpcs":
            if req.method == "POST":
                body = json.loads(req.content)
                vpcs.append({"id": "vpc-1", "region": body["region"], "description": body["description"],
                             "v4_subnet": "10.40.96.0", "v4_subnet_mask": 20})
                return httpx.Response(201, json={"vpc": vpcs[-1]})
            return httpx.Response(200, json={"vpcs": vpcs, "meta": {"links": {"next": ""}}})
        if req.method == "POST" and req.url.path == "/v2/bare-metals":
            body = json.loads(req.content)
            posts.append(body)
            assert body["plan"].endswith("mi355x-gpu") and body["attach_vpc"] == ["vpc-1"]
            ud = base64.b64decode(body["user_data"]).decode()
            assert "dstack-shim" in ud and "ufw allow from 10.40.96.0/20" in ud
            return httpx.Response(202, json={"bare_metal": {"id": f"bm-{len(posts)}"}})
        if req.method == "GET" and req.url.path.endswith("/vpcs"):
            return httpx.Response(200, json={"vpcs": [{"id": "vpc-1", "ip_address": "10.40.96.3"}]})
        if req.method == "GET" and req.url.path.startswith("/v2/bare-metals/bm-"):
            return httpx.Response(200, json={"bare_metal": {"status": state["status"], "main_ip": "5.5.5.5"}})
        if req.method == "DELETE":
            return httpx.Response(204)
        return httpx.Response(404)

    c = compute_class(BackendType.VULTR)({}, {"api_key": "vk"}, _client(handler))
    offer = _offer(c, "MI355X:8")
    assert offer.instance.resources.gpus[0].name == "MI355X" and len(offer.instance.resources.gpus) == 8
    jpd = c.create_instance(offer, CFG)
    c.update_provisioning_data(jpd)
    assert jpd.hostname is None  # not active yet
    state["status"] = "active"
    c.update_provisioning_data(jpd)
    assert jpd.hostname == "5.5.5.5" and jpd.username == "root" and jpd.internal_ip == "10.40.96.3"
    c.create_instance(offer, CFG)  # a second node of the cluster: same VPC, no new one
    assert len(vpcs) == 1 and [p["attach_vpc"] for p in posts] == [["vpc-1"], ["vpc-1"]]
    assert posts[0]["os_id"] == 1743
    c.terminate_instance(jpd.instance_id, jpd.region, jpd.backend_data)
    # a ROCm marketplace image for the bare-metal plans
    c2 = compute_class(BackendType.VULTR)({"images": {"bare_metal": "amd-rocm"}}, {"api_key": "vk"}, _client(handler))
    c2.create_instance(offer, CFG)
    assert posts[-1]["image_id"] == "amd-rocm" and "os_id" not in posts[-1]


def test_nebius_service_account_key_exchanged_for_cached_iam_token(rsa_pem):
    """A service-account authorized key is turned into an IAM token with a PS256 JWT; the token
    is cached across calls."""
    exchanges, seen = [], []

    def handler(req):
        if req.url.host == "iam.api.nebius.cloud":
            jwt = json.loads(req.content)["jwt"]
            head, claims, sig = jwt.split(".")
            pad = lambda x: x + "=" * (-len(x) % 4)  # noqa: E731
            h = json.loads(base64.urlsafe_b64decode(pad(head)))
            c = json.loads(base64.urlsafe_b64decode(pad(claims)))
            assert h == {"typ": "JWT", "alg": "PS256", "kid": "key-1"} and c["iss"] == "sa-1"
            assert c["aud"].endswith("/iam/v1/tokens") and c["exp"] > c["iat"]
            assert len(base64.urlsafe_b64decode(pad(sig))) >= 256  # an RSA-2048+ signature
            exchanges.append(jwt)
            return httpx.Response(200, json={"iamToken": "t-123", "expiresAt": "2099-01-01T00:00:00Z"})
        seen.append(req.headers["authorization"])
        return httpx.Response(200, json={"instances": []})

    key = json.dumps({"id": "key-1", "service_account_id": "sa-1", "private_key": rsa_pem})
    c = compute_class(BackendType.NEBIUS)({"folder_id": "f"}, {"type": "service_account", "data": key},
                                          _client(handler))
    c.check_credentials()
    c.check_credentials()
    assert len(exchanges) == 1 and seen == ["Bearer t-123", "Bearer t-123"]


# ---- RunPod (MI300X containers) ----------------------------------------------------------------
def test_runpod_pod_lifecycle():
    seen = []

    def handler(req):
        q = json.loads(req.content)
        seen.append(q["query"].split("(")[0].split()[-1] if "mutation" in q["query"] else "query")
        if "podFindAndDeployOnDemand" in q["query"]:
            inp = q["variables"]["input"]
            assert inp["gpuTypeId"] == "AMD Instinct MI300X OAM" and "dstack-runner" in inp["dockerArgs"]
            return httpx.Response(200, json={"data": {"podFindAndDeployOnDemand": {"id": "pod1", "machineId": "m"}}})
        if "pod(input" in q["query"]:
            return httpx.Response(200, json={"data": {"pod": {"id": "pod1", "runtime": {"ports": [
                {"ip": "7.7.7.7", "isIpPublic": True, "privatePort": 10022, "publicPort": 40022, "type": "tcp"}]}}}})
        if "podTerminate" in q["query"]:
            return httpx.Response(200, json={"data": {"podTerminate": None}})
        return httpx.Response(200, json={"errors": [{"message": "unexpected"}]})

    from types import SimpleNamespace

    c = compute_class(BackendType.RUNPOD)({}, {"api_key": "rk"}, _client(handler))
    offer = _offer(c, "MI300X:1")
    run = SimpleNamespace(run_spec=SimpleNamespace(run_name="r", ssh_key_pub="ssh-ed25519 USER"))
    job = SimpleNamespace(job_spec=SimpleNamespace(job_num=0, image_name=None))
    jpd = c.run_job(run, job, offer, "ssh-ed25519 PROJECT", "", [])
    assert jpd.instance_id == "pod1" and not jpd.dockerized
    c.update_provisioning_data(jpd)
    assert (jpd.hostname, jpd.ssh_port) == ("7.7.7.7", 40022)
    c.terminate_instance("pod1", jpd.region)


def test_runpod_no_capacity():
    def handler(req):
        return httpx.Response(200, json={"errors": [{"message": "There are no longer any instances available"}]})

    from types import SimpleNamespace

    c = compute_class(BackendType.RUNPOD)({}, {"api_key": "rk"}, _client(handler))
    run = SimpleNamespace(run_spec=SimpleNamespace(run_name="r", ssh_key_pub=""))
    job = SimpleNamespace(job_spec=SimpleNamespace(job_num=0, image_name=None))
    with pytest.raises(NoCapacityError):
        c.run_job(run, job, _offer(c, "MI300X:1"), "ssh-ed25519 K", "", [])


# ---- Lambda / DataCrunch / Cudo ----------------------------------------------------------------
def test_lambda_launch_registers_key_once_by_fingerprint():
    """The instance's key is added under a name derived from its fingerprint; a key already in the
    account (any name) is reused; an insufficient-capacity answer is a NoCapacityError."""
    from dstack_amd.core.backends.clouds.common import ssh_key_fingerprint

    keys, launches = [{"name": "someone-elses", "public_key": "ssh-rsa BBBB other"}], []
    state = {"capacity": True}

    def handler(req):
        p = req.url.path
        if p.endswith("/ssh-keys") and req.method == "GET":
            return httpx.Response(200, json={"data": keys})
        if p.endswith("/ssh-keys"):
            keys.append(json.loads(req.content))
            return httpx.Response(200, json={"data": {}})
        if p.endswith("/launch"):
            if not state["capacity"]:
                return httpx.Response(400, json={"error": {"code": "instance-operations/launch/insufficient-capacity"}})
            launches.append(json.loads(req.content))
            return httpx.Response(200, json={"data": {"instance_ids": ["L1"]}})
        if p.endswith("/instances/L1"):
            return httpx.Response(200, json={"data": {"status": "active", "ip": "9.9.9.9"}})
        if p.endswith("/terminate"):
            return httpx.Response(200, json={"data": {}})
        return httpx.Response(404)

    c = compute_class(BackendType.LAMBDA)({}, {"api_key": "lk"}, _client(handler))
    jpd = c.create_instance(_offer(c, "H100:8"), CFG)
    c.update_provisioning_data(jpd)
    assert jpd.hostname == "9.9.9.9" and len(keys) == 2
    added = keys[1]
    assert added["name"].startswith("dstack-") and ssh_key_fingerprint(added["public_key"]) == \
        ssh_key_fingerprint(CFG.ssh_keys[0].public)
    c.create_instance(_offer(c, "H100:8"), CFG)  # same key again: reused, not re-added
    assert len(keys) == 2 and launches[0]["ssh_key_names"] == launches[1]["ssh_key_names"] == [added["name"]]
    c.terminate_instance("L1", jpd.region)
    state["capacity"] = False
    with pytest.raises(NoCapacityError):
        c.create_instance(_offer(c, "H100:8"), CFG)


def test_datacrunch_oauth_token_cached_and_account_objects_reused():
    tokens, created = [], []
    scripts, sshkeys = [], [{"id": "key-0", "name": "mine", "key": CFG.ssh_keys[0].public}]

    def handler(req):
        if req.url.path.endswith("/oauth2/token"):
            tokens.append(1)
            return httpx.Response(200, json={"access_token": "T", "expires_in": 3600})
        assert req.headers["authorization"] == "Bearer T"
        if req.url.path.endswith("/scripts"):
            if req.method == "GET":
                return httpx.Response(200, json=scripts)
            body = json.loads(req.content)
            scripts.append({"id": f"script-{len(scripts) + 1}", **body})
            created.append("script")
            return httpx.Response(200, text=f'"script-{len(scripts)}"')
        if req.url.path.endswith("/sshkeys"):
            if req.method == "GET":
                return httpx.Response(200, json=sshkeys)
            created.append("key")
            return httpx.Response(200, text='"key-new"')
        if req.url.path.endswith("/instances") and req.method == "POST":
            body = json.loads(req.content)
            assert body["ssh_key_ids"] == ["key-0"] and body["startup_script_id"] == "script-1"
            return httpx.Response(200, text='"inst-1"')
        return httpx.Response(200, json={"status": "running", "ip": "1.2.3.4"})

    c = compute_class(BackendType.DATACRUNCH)({}, {"client_id": "a", "client_secret": "b"}, _client(handler))
    jpd = c.create_instance(_offer(c, "H100:8"), CFG)
    c.update_provisioning_data(jpd)
    assert jpd.instance_id == "inst-1" and jpd.hostname == "1.2.3.4"
    c.create_instance(_offer(c, "H100:8"), CFG)  # the same script content and key: both reused
    assert created == ["script"] and len(tokens) == 1


# ---- GCP / OCI signing with a real RSA key ---------------------------------------------------
@pytest.fixture(scope="module")
def rsa_pem(tmp_path_factory):
    p = tmp_path_factory.mktemp("k") / "key.pem"
    subprocess.run(["openssl", "genrsa", "-out", str(p), "2048"], check=True, capture_output=True)
    return p.read_text()


def test_gcp_jwt_token_and_insert(rsa_pem):
    def handler(req):
        if req.url.host == "oauth2.googleapis.com":
            form = dict(urllib.parse.parse_qsl(req.content.decode()))
            assert form["grant_type"].endswith("jwt-bearer")
            assert len(form["assertion"].split(".")) == 3
            return httpx.Response(200, json={"access_token": "G", "expires_in": 3600})
        assert req.headers["authorization"] == "Bearer G"
        if req.method == "POST":
            body = json.loads(req.content)
            assert body["scheduling"]["onHostMaintenance"] == "TERMINATE"
            return httpx.Response(200, json={"name": "op"})
        return httpx.Response(200, json={"status": "RUNNING", "networkInterfaces": [
            {"networkIP": "10.1.1.1", "accessConfigs": [{"natIP": "34.1.1.1"}]}]})

    sa = {"client_email": "sa@p.iam.gserviceaccount.com", "private_key": rsa_pem, "project_id": "p"}
    c = compute_class(BackendType.GCP)({}, {"data": json.dumps(sa)}, _client(handler))
    jpd = c.create_instance(_offer(c, "H100:8"), CFG)
    c.update_provisioning_data(jpd)
    assert jpd.hostname == "34.1.1.1"


def test_oci_http_signature(rsa_pem):
    def handler(req):
        auth = req.headers["authorization"]
        assert auth.startswith('Signature version="1",keyId="ten/usr/fp",algorithm="rsa-sha256"')
        if req.method == "POST":
            assert 'headers="(request-target) date host x-content-sha256 content-type content-length"' in auth
            body = json.loads(req.content)
            assert body["shape"] == "BM.GPU.MI300X.8"
            assert body["sourceDetails"]["imageId"] == "ocid1.image.ubuntu"  # looked up, never ""
            # the tenancy's real AD name that offers the shape (not "<region>-AD-1")
            assert body["availabilityDomain"] == "Uocm:US-CHICAGO-1-AD-2"
            assert body["createVnicDetails"]["subnetId"] == "ocid1.subnet.pre"  # the configured subnet
            return httpx.Response(200, json={"id": "ocid1.instance"})
        if req.url.host.startswith("identity.") and req.url.path.endswith("/availabilityDomains"):
            return httpx.Response(200, json=[{"name": "Uocm:US-CHICAGO-1-AD-1"}, {"name": "Uocm:US-CHICAGO-1-AD-2"}])
        if req.url.path.endswith("/shapes"):
            ad = dict(urllib.parse.parse_qsl(req.url.query.decode()))["availabilityDomain"]
            shapes = ["VM.Standard.E4.Flex"] + (["BM.GPU.MI300X.8"] if ad.endswith("AD-2") else [])
            return httpx.Response(200, json=[{"shape": x} for x in shapes])
        if req.url.path.endswith("/images"):
            q = dict(urllib.parse.parse_qsl(req.url.query.decode()))
            assert q["shape"] == "BM.GPU.MI300X.8" and q["operatingSystemVersion"] == "22.04"
            return httpx.Response(200, json=[{"id": "ocid1.image.ubuntu"}, {"id": "ocid1.image.older"}])
        if "vnicAttachments" in str(req.url):
            return httpx.Response(200, json=[{"vnicId": "v1"}])
        if "/vnics/" in req.url.path:
            return httpx.Response(200, json={"publicIp": "140.1.1.1", "privateIp": "10.0.0.9"})
        return httpx.Response(200, json={"lifecycleState": "RUNNING"})

    c = compute_class(BackendType.OCI)({"compartment_id": "comp"}, {"tenancy": "ten", "user": "usr",
                                                                      "fingerprint": "fp", "key_content": rsa_pem},
                                       _client(handler))
    offer = _offer(c, "MI300X:8")
    c.config["subnet_ids"] = {offer.region: "ocid1.subnet.pre"}
    jpd = c.create_instance(offer, CFG)
    c.update_provisioning_data(jpd)
    assert jpd.hostname == "140.1.1.1"


# ---- Kubernetes -------------------------------------------------------------------------------
def test_kubernetes_offers_and_pod():
    created = []

    def handler(req):
        p = req.url.path
        if p == "/api/v1/nodes":
            return httpx.Response(200, json={"items": [{"metadata": {"name": "mi355x-node", "labels": {
                "amd.com/gpu.product-name": "AMD Instinct MI355 OAM"}}, "status": {"allocatable": {
                    "cpu": "256", "memory": "3000Gi", "amd.com/gpu": "8", "ephemeral-storage": "10Ti"}}}]})
        if req.method == "POST":
            body = json.loads(req.content)
            created.append(body["kind"])
            if body["kind"] == "Pod" and body["metadata"]["name"] != "dstack-ssh-jump":
                lim = body["spec"]["containers"][0]["resources"]["limits"]
                assert lim["amd.com/gpu"] == "8"
            if body["kind"] == "Service" and body["spec"]["type"] == "NodePort":
                return httpx.Response(201, json={"spec": {"ports": [{"nodePort": 30022}]}})
            return httpx.Response(201, json=body)
        if p.endswith("/services/dstack-ssh-jump"):
            return httpx.Response(404)
        if "/services/" in p:
            return httpx.Response(200, json={"spec": {"clusterIP": "10.96.0.5"}})
        if "/pods/" in p:
            return httpx.Response(200, json={"status": {"phase": "Running", "podIP": "10.244.0.7"}})
        return httpx.Response(404)

    from types import SimpleNamespace

    kubeconfig = {"data": json.dumps({"current-context": "c", "contexts": [{"name": "c", "context": {
        "cluster": "k", "user": "u"}}], "clusters": [{"name": "k", "cluster": {"server": "https://k8s.example:6443"}}],
        "users": [{"name": "u", "user": {"token": "tok"}}]})}
    c = compute_class(BackendType.KUBERNETES)({"kubeconfig": kubeconfig}, {}, _client(handler))
    offers = c.get_offers(Requirements(resources=ResourcesSpec.model_validate({"gpu": "MI355X:8"})))
    assert len(offers) == 1 and offers[0].instance.resources.gpus[0].name == "MI355X"
    run = SimpleNamespace(run_spec=SimpleNamespace(run_name="r", ssh_key_pub=""))
    job = SimpleNamespace(job_spec=SimpleNamespace(job_num=0, replica_num=0, image_name=None))
    jpd = c.run_job(run, job, offers[0], "ssh-ed25519 K", "", [])
    assert jpd.ssh_proxy.port == 30022 and jpd.ssh_proxy.hostname == "k8s.example"
    c.update_provisioning_data(jpd)
    assert jpd.hostname == "10.96.0.5"
    assert created.count("Pod") == 2 and created.count("Service") == 2


def test_every_cloud_backend_plans_offers():
    for bt in BackendType:
        cls = compute_class(bt)
        if cls is None or bt == BackendType.KUBERNETES:
            continue
        c = cls({}, {}, _client(lambda req: httpx.Response(500)))
        assert isinstance(c.get_offers(None), list)
        assert re.match(r"^[a-z]+$", c.TYPE.value)


# ---- Docker registry introspection -------------------------------------------------------------
def test_registry_image_config_with_token_challenge():
    from dstack_amd.server.services.docker import RegistryClient, parse_image_name

    assert parse_image_name("ubuntu").repository == "library/ubuntu"
    assert parse_image_name("rocm/pytorch:latest").reference == "latest"
    r = parse_image_name("ghcr.io/org/img@sha256:abc")
    assert (r.registry, r.repository, r.reference) == ("ghcr.io", "org/img", "sha256:abc")

    def handler(req):
        if req.url.host == "auth.docker.io":
            assert req.url.params["scope"] == "repository:rocm/vllm:pull"
            return httpx.Response(200, json={"token": "T"})
        if req.headers.get("authorization") != "Bearer T":
            return httpx.Response(401, headers={"www-authenticate": 'Bearer realm="https://auth.docker.io/token",'
                                                                     'service="registry.docker.io",'
                                                                     'scope="repository:rocm/vllm:pull"'})
        if req.url.path.endswith("/manifests/latest"):
            return httpx.Response(200, json={"manifests": [
                {"digest": "sha256:arm", "platform": {"os": "linux", "architecture": "arm64"}},
                {"digest": "sha256:amd", "platform": {"os": "linux", "architecture": "amd64"}}]})
        if req.url.path.endswith("/manifests/sha256:amd"):
            return httpx.Response(200, json={"config": {"digest": "sha256:cfg"}})
        if req.url.path.endswith("/blobs/sha256:cfg"):
            return httpx.Response(200, json={"config": {"User": "1000:1000", "Entrypoint": ["python3", "-m", "vllm"],
                                                        "Cmd": ["serve"], "Env": ["PATH=/usr/bin"]}})
        return httpx.Response(404)

    rc = RegistryClient(_client(handler))
    cfg = rc.get_image_config("rocm/vllm")
    assert cfg.user == "1000:1000" and cfg.entrypoint == ["python3", "-m", "vllm"] and cfg.cmd == ["serve"]


def test_registry_refusal_fails_submission_unreachable_registry_does_not(monkeypatch):
    """An unknown image (registry answers 404) fails the job spec with a client error, as in the
    reference; a registry that cannot be reached only skips the lookup."""
    from dstack_amd.core.errors import DockerRegistryError, ServerClientError
    from dstack_amd.core.models.configurations import parse_run_configuration
    from dstack_amd.server.services import docker as docker_mod
    from dstack_amd.server.services.jobs import configurators

    rc = docker_mod.RegistryClient(_client(lambda req: httpx.Response(404)))
    with pytest.raises(DockerRegistryError) as ei:
        rc.get_image_config("rocm/does-not-exist:1")
    assert ei.value.status == 404
    conf = parse_run_configuration({"type": "task", "image": "rocm/does-not-exist:1"})
    monkeypatch.setattr(docker_mod, "_client", rc)
    with pytest.raises(ServerClientError, match="Error pulling configuration for image"):
        configurators._image_config(conf)

    def unreachable(req):
        raise httpx.ConnectError("no route to host")

    monkeypatch.setattr(docker_mod, "_client", docker_mod.RegistryClient(_client(unreachable)))
    assert configurators._image_config(conf) is None


def _aws_vpc_handler(calls, capacity_fail_az=None, efa=True, reservation_type="capacity-block"):
    def handler(req: httpx.Request):
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        a = form["Action"]
        calls.append(form)
        if a == "DescribeVpcs":
            assert form["Filter.1.Value.1"] == "dstack-vpc"
            return httpx.Response(200, text=_xml("<vpcSet><item><vpcId>vpc-9</vpcId></item></vpcSet>"))
        if a == "DescribeSubnets":
            if "NextToken" not in form:  # page 1 of 2
                return httpx.Response(200, text=_xml(
                    "<subnetSet><item><subnetId>sn-b</subnetId><availabilityZone>us-east-1b</availabilityZone>"
                    "<mapPublicIpOnLaunch>false</mapPublicIpOnLaunch></item></subnetSet><nextToken>p2</nextToken>"))
            return httpx.Response(200, text=_xml(
                "<subnetSet><item><subnetId>sn-a</subnetId><availabilityZone>us-east-1a</availabilityZone>"
                "<mapPublicIpOnLaunch>false</mapPublicIpOnLaunch></item></subnetSet>"))
        if a == "DescribeInstanceTypes":
            info = ("<networkInfo><efaSupported>true</efaSupported><maximumNetworkCards>32</maximumNetworkCards>"
                    "<efaInfo><maximumEfaInterfaces>32</maximumEfaInterfaces></efaInfo></networkInfo>") if efa else \
                "<networkInfo><efaSupported>false</efaSupported></networkInfo>"
            return httpx.Response(200, text=_xml(f"<instanceTypeSet><item>{info}</item></instanceTypeSet>"))
        if a == "DescribeCapacityReservations":
            return httpx.Response(200, text=_xml(
                "<capacityReservationSet><item><state>active</state><availabilityZone>us-east-1b</availabilityZone>"
                f"<reservationType>{reservation_type}</reservationType><instanceType>p5.48xlarge</instanceType>"
                "</item></capacityReservationSet>"))
        if a == "DescribeImages":
            return httpx.Response(200, text=_xml("<imagesSet><item><imageId>ami-1</imageId></item></imagesSet>"))
        if a == "DescribeSecurityGroups":
            assert form.get("Filter.2.Value.1") == "vpc-9"
            return httpx.Response(200, text=_xml("<securityGroupInfo><item><groupId>sg-9</groupId></item>"
                                                 "</securityGroupInfo>"))
        if a == "RunInstances":
            if form.get("NetworkInterface.1.SubnetId") == capacity_fail_az:
                return httpx.Response(500, text=_xml("<Errors><Error><Code>InsufficientInstanceCapacity</Code>"
                                                     "<Message>no</Message></Error></Errors>"))
            return httpx.Response(200, text=_xml("<instancesSet><item><instanceId>i-9</instanceId></item>"
                                                 "</instancesSet>"))
        if a == "DescribeInstances":
            return httpx.Response(200, text=_xml("<reservationSet><item><instancesSet><item><instanceState><name>"
                                                 "running</name></instanceState><ipAddress>3.3.3.3</ipAddress>"
                                                 "<privateIpAddress>10.9.0.5</privateIpAddress></item></instancesSet>"
                                                 "</item></reservationSet>"))
        return httpx.Response(400, text=_xml(f"<Errors><Error><Code>Unexpected{a}</Code></Error></Errors>"))
    return handler


def test_aws_named_vpc_private_efa_cluster_interfaces():
    """p5.48xlarge in a named VPC without public IPs: all 32 EFA cards requested (every 4th ``efa``,
    the rest ``efa-only``), subnets from a paginated DescribeSubnets tried one AZ at a time (the first
    AZ has no capacity), and the host reached on its private address."""
    calls = []
    c = compute_class(BackendType.AWS)({"vpc_name": "dstack-vpc", "public_ips": False},
                                       {"access_key": "AK", "secret_key": "SK"},
                                       _client(_aws_vpc_handler(calls, capacity_fail_az="sn-a")))
    offer = _offer(c, "H100:8")
    assert offer.instance.name == "p5.48xlarge"
    jpd = c.create_instance(offer, CFG)
    runs = [f for f in calls if f["Action"] == "RunInstances"]
    assert [r["NetworkInterface.1.SubnetId"] for r in runs] == ["sn-a", "sn-b"]  # us-east-1a first, then 1b
    r = runs[-1]
    assert "SecurityGroupId.1" not in r and r["NetworkInterface.1.SecurityGroupId.1"] == "sg-9"
    assert r["NetworkInterface.1.InterfaceType"] == "efa" and r["NetworkInterface.1.AssociatePublicIpAddress"] == "false"
    cards = {int(r[f"NetworkInterface.{n}.NetworkCardIndex"]): r[f"NetworkInterface.{n}.InterfaceType"]
             for n in range(2, 33)}
    assert sorted(cards) == list(range(1, 32))
    assert [k for k, v in cards.items() if v == "efa"] == [4, 8, 12, 16, 20, 24, 28]
    assert r["TagSpecification.1.Tag.3.Key"] == "dstack_project"
    c.update_provisioning_data(jpd)
    assert jpd.hostname == "10.9.0.5"  # private address


def test_aws_capacity_block_reservation_pins_zone_and_market():
    from dstack_amd.core.models.instances import InstanceConfiguration, SSHKey

    calls = []
    c = compute_class(BackendType.AWS)({"vpc_name": "dstack-vpc"}, {"access_key": "AK", "secret_key": "SK"},
                                       _client(_aws_vpc_handler(calls, efa=False)))
    cfg = InstanceConfiguration(project_name="main", instance_name="r-0", user="admin", reservation="cr-123",
                                ssh_keys=[SSHKey(public="ssh-ed25519 AAAA k")])
    c2 = compute_class(BackendType.AWS)({"vpc_name": "dstack-vpc", "public_ips": False},
                                        {"access_key": "AK", "secret_key": "SK"},
                                        _client(_aws_vpc_handler(calls, efa=False)))
    c2.create_instance(_offer(c, "H100:8"), cfg)
    r = [f for f in calls if f["Action"] == "RunInstances"][-1]
    assert r["InstanceMarketOptions.MarketType"] == "capacity-block"
    assert r["NetworkInterface.1.SubnetId"] == "sn-b"  # the reservation's zone
    assert r["CapacityReservationSpecification.CapacityReservationTarget.CapacityReservationId"] == "cr-123"
    assert r["NetworkInterface.1.InterfaceType"] == "interface"


# ---- gateways and volumes on GCP / Azure / Kubernetes --------------------------------------------
def _gw_conf(backend, region):
    from dstack_amd.core.models.gateways import GatewayComputeConfiguration

    return GatewayComputeConfiguration(project_name="main", instance_name="gw-1", backend=backend, region=region,
                                       public_ip=True, ssh_key_pub="ssh-rsa AAA gw")


def test_gcp_gateway_firewall_insert_and_terminate(rsa_pem, monkeypatch):
    monkeypatch.setattr("time.sleep", lambda *_: None)
    seen = []

    def handler(req):
        if req.url.host == "oauth2.googleapis.com":
            return httpx.Response(200, json={"access_token": "G", "expires_in": 3600})
        seen.append((req.method, req.url.path))
        if req.url.path.endswith("/global/firewalls"):
            body = json.loads(req.content)
            assert body["targetTags"] == ["dstack-gateway"] and body["allowed"][0]["ports"] == ["22", "80", "443"]
            return httpx.Response(409, json={"error": "exists"})
        if req.method == "POST" and req.url.path.endswith("/instances"):
            body = json.loads(req.content)
            assert body["tags"]["items"] == ["dstack-gateway"] and "e2-small" in body["machineType"]
            ud = body["metadata"]["items"][0]["value"]
            assert ud.startswith("#cloud-config") and "dstack_amd-gateway-" in ud
            return httpx.Response(200, json={"status": "DONE", "selfLink": "https://op/1"})
        if req.method == "DELETE":
            return httpx.Response(200, json={"status": "DONE"})
        return httpx.Response(200, json={"status": "RUNNING", "networkInterfaces": [
            {"networkIP": "10.1.1.2", "accessConfigs": [{"natIP": "34.2.2.2"}]}]})

    sa = {"client_email": "sa@p.iam.gserviceaccount.com", "private_key": rsa_pem, "project_id": "p"}
    c = compute_class(BackendType.GCP)({}, {"data": json.dumps(sa)}, _client(handler))
    gpd = c.create_gateway(_gw_conf(BackendType.GCP, "us-central1"))
    assert gpd.ip_address == "34.2.2.2" and json.loads(gpd.backend_data)["zone"] == "us-central1-a"
    c.terminate_gateway(gpd.instance_id, _gw_conf(BackendType.GCP, "us-central1"), gpd.backend_data)
    assert seen[-1] == ("DELETE", "/compute/v1/projects/p/zones/us-central1-a/instances/gw-1")


def test_gcp_persistent_disk_volume_lifecycle(rsa_pem, monkeypatch):
    import datetime as dt
    import uuid

    from dstack_amd.core.models.volumes import Volume, VolumeConfiguration, VolumeStatus

    monkeypatch.setattr("time.sleep", lambda *_: None)
    state = {"users": [], "polls": 0}
    calls = []

    def handler(req):
        if req.url.host == "oauth2.googleapis.com":
            return httpx.Response(200, json={"access_token": "G", "expires_in": 3600})
        calls.append((req.method, req.url.path + ("?" + req.url.query.decode() if req.url.query else "")))
        if req.url.host == "op":  # operation polling: RUNNING once, then DONE
            state["polls"] += 1
            return httpx.Response(200, json={"status": "DONE"})
        if req.method == "POST" and req.url.path.endswith("/disks"):
            body = json.loads(req.content)
            assert body["sizeGb"] == "200" and body["type"].endswith("diskTypes/pd-balanced")
            return httpx.Response(200, json={"status": "RUNNING", "selfLink": "https://op/disk"})
        if req.url.path.endswith("/attachDisk"):
            body = json.loads(req.content)
            assert body["deviceName"] == body["source"].rsplit("/", 1)[1]
            state["users"] = ["https://compute/projects/p/zones/us-central1-a/instances/inst-7"]
            return httpx.Response(200, json={"status": "DONE"})
        if "/detachDisk" in req.url.path:
            state["users"] = []
            return httpx.Response(200, json={"status": "DONE"})
        if req.method == "DELETE":
            return httpx.Response(200, json={"status": "DONE"})
        return httpx.Response(200, json={"name": "data-x", "sizeGb": "200", "users": state["users"]})

    sa = {"client_email": "sa@p.iam.gserviceaccount.com", "private_key": rsa_pem, "project_id": "p"}
    c = compute_class(BackendType.GCP)({}, {"data": json.dumps(sa)}, _client(handler))
    vol = Volume(id=uuid.uuid4(), name="data", project_name="main", external=False, status=VolumeStatus.SUBMITTED,
                 created_at=dt.datetime.now(dt.timezone.utc),
                 configuration=VolumeConfiguration(backend=BackendType.GCP, region="us-central1", size=200))
    vpd = c.create_volume(vol)
    assert state["polls"] == 1 and vpd.availability_zone == "us-central1-a" and vpd.size_gb == 200
    vol = vol.model_copy(update={"volume_id": vpd.volume_id, "provisioning_data": vpd})
    vad = c.attach_volume(vol, "inst-7")
    assert vad.device_name == vpd.volume_id  # /dev/disk/by-id/google-<device name> on the host
    assert not c.is_volume_detached(vol, "inst-7")
    c.detach_volume(vol, "inst-7")
    assert c.is_volume_detached(vol, "inst-7")
    c.delete_volume(vol)
    assert calls[-1][0] == "DELETE" and calls[-1][1].endswith(f"/disks/{vpd.volume_id}")


def test_azure_creates_network_and_gateway_with_http_nsg(monkeypatch):
    monkeypatch.setattr("time.sleep", lambda *_: None)
    deployed = {}

    def handler(req):
        if req.url.host == "login.microsoftonline.com":
            return httpx.Response(200, json={"access_token": "A", "expires_in": 3600})
        if req.method == "PUT" and "/deployments/" in req.url.path:
            deployed["tpl"] = json.loads(req.content)["properties"]["template"]
            return httpx.Response(201, json={})
        if req.method == "PUT":
            return httpx.Response(200, json={})
        if "/deployments/" in req.url.path:
            return httpx.Response(200, json={"properties": {"provisioningState": "Running"}})
        if "publicIPAddresses" in req.url.path and req.method == "GET":
            return httpx.Response(200, json={"properties": {"ipAddress": "20.1.1.1"}})
        return httpx.Response(200, json={})

    c = compute_class(BackendType.AZURE)({"subscription_id": "sub", "tenant_id": "t"},
                                         {"client_id": "c", "client_secret": "s"}, _client(handler))
    gpd = c.create_gateway(_gw_conf(BackendType.AZURE, "eastus"))
    assert gpd.ip_address == "20.1.1.1"
    res = {r["type"].split("/")[-1] + ":" + r["name"]: r for r in deployed["tpl"]["resources"]}
    assert "virtualNetworks:dstack-vnet-eastus" in res and "networkSecurityGroups:dstack-nsg-eastus" in res
    ports = [r["properties"]["destinationPortRange"] for r in res["networkSecurityGroups:gw-1-nsg"]["properties"]
             ["securityRules"]]
    assert ports == ["22", "80", "443"]
    nic = res["networkInterfaces:gw-1-nic"]
    assert any("dstack-vnet-eastus" in d for d in nic["dependsOn"]) and "networkSecurityGroup" in nic["properties"]
    # a VM deployment declares the VNet it joins too (nothing has to pre-exist)
    c2 = compute_class(BackendType.AZURE)({"subscription_id": "sub", "tenant_id": "t"},
                                          {"client_id": "c", "client_secret": "s"}, _client(handler))
    c2.create_instance(_offer(c2, "MI300X:8"), CFG)
    names = [r["name"] for r in deployed["tpl"]["resources"]]
    assert "dstack-vnet-eastus" in names or any(n.startswith("dstack-vnet-") for n in names)


def _kube_compute(handler, **cfg):
    kubeconfig = {"data": json.dumps({"current-context": "c", "contexts": [{"name": "c", "context": {
        "cluster": "k", "user": "u"}}], "clusters": [{"name": "k", "cluster": {"server": "https://k8s.example:6443"}}],
        "users": [{"name": "u", "user": {"token": "tok"}}]})}
    return compute_class(BackendType.KUBERNETES)({"kubeconfig": kubeconfig, "gateway_lb_wait_s": 0, **cfg}, {},
                                                 _client(handler))


def test_kubernetes_gateway_pod_and_load_balancer():
    polls = {"n": 0}
    created, deleted = [], []

    def handler(req):
        if req.method == "POST":
            body = json.loads(req.content)
            created.append(body)
            return httpx.Response(201, json=body)
        if req.method == "DELETE":
            deleted.append(req.url.path)
            return httpx.Response(200, json={})
        polls["n"] += 1
        ing = [{"hostname": "gw.elb.example"}] if polls["n"] >= 3 else []
        return httpx.Response(200, json={"status": {"loadBalancer": {"ingress": ing}}})

    c = _kube_compute(handler)
    gpd = c.create_gateway(_gw_conf(BackendType.KUBERNETES, "default"))
    assert gpd.ip_address == "gw.elb.example" and json.loads(gpd.backend_data)["ssh_user"] == "root"
    pod, svc = created
    script = pod["spec"]["containers"][0]["args"][1]
    assert "update.sh" in script and script.rstrip().endswith("exec /usr/sbin/sshd -D")
    assert svc["spec"]["type"] == "LoadBalancer" and [p["port"] for p in svc["spec"]["ports"]] == [22, 80, 443]
    c.terminate_gateway(gpd.instance_id, _gw_conf(BackendType.KUBERNETES, "default"), gpd.backend_data)
    assert deleted == ["/api/v1/namespaces/default/services/gw-1-service", "/api/v1/namespaces/default/pods/gw-1"]


def test_kubernetes_gateway_without_load_balancer_is_cleaned_up():
    from dstack_amd.core.errors import ComputeError

    deleted = []

    def handler(req):
        if req.method == "POST":
            return httpx.Response(201, json={})
        if req.method == "DELETE":
            deleted.append(req.url.path)
            return httpx.Response(200, json={})
        return httpx.Response(200, json={"status": {"loadBalancer": {}}})

    c = _kube_compute(handler, gateway_lb_wait_tries=3)
    with pytest.raises(ComputeError, match="LoadBalancer"):
        c.create_gateway(_gw_conf(BackendType.KUBERNETES, "default"))
    assert len(deleted) == 2


def test_gateway_scripts_survive_shell_and_cloud_init_quoting(tmp_path):
    """The scripts reach the host byte for byte: through sh -c (Kubernetes args) and through
    cloud-init's YAML (runcmd items are JSON-quoted YAML strings)."""
    import yaml

    from dstack_amd.core.backends.clouds.gateway_boot import gateway_cloud_init
    from dstack_amd.proxy.gateway import packaging

    for content, path in ((packaging.UPDATE_SH, "update.sh"), (packaging.RESTART_SH, "restart"),
                          (packaging.SYSTEMD_UNIT, "unit")):
        cmd = packaging.write_file_command(content, str(tmp_path / path))
        subprocess.run(["sh", "-c", cmd], check=True)
        assert (tmp_path / path).read_text() == content
    ci = yaml.safe_load(gateway_cloud_init(_gw_conf(BackendType.AWS, "us-east-1")))
    writes = [c for c in ci["runcmd"] if "base64 -d >" in c]
    assert len(writes) == 2
    for c in writes:
        target = c.split("> ", 1)[1].split(" ")[0]
        local = tmp_path / os.path.basename(target)
        subprocess.run(["sh", "-c", c.replace(target, str(local))], check=True)
    assert (tmp_path / "update.sh").read_text() == packaging.UPDATE_SH
    assert (tmp_path / "dstack-gateway.service").read_text() == packaging.SYSTEMD_UNIT


def test_capability_lists_match_implementations():
    """Every backend advertised for gateways / volumes implements the calls (no base-class
    NotImplementedError behind an advertised capability)."""
    from dstack_amd.core.backends.base import Compute
    from dstack_amd.core.models.backends import BACKENDS_WITH_GATEWAY_SUPPORT, BACKENDS_WITH_VOLUMES_SUPPORT

    def cls_of(bt):
        if bt == BackendType.LOCAL:
            from dstack_amd.core.backends.local import LocalCompute
            return LocalCompute
        if bt == BackendType.REMOTE:
            from dstack_amd.core.backends.remote import RemoteCompute
            return RemoteCompute
        return compute_class(bt)

    for bt in BACKENDS_WITH_GATEWAY_SUPPORT:
        if bt == BackendType.LOCAL:
            continue  # local gateways run in-process (services.gateways.LocalGatewayProcess)
        cls = cls_of(bt)
        for m in ("create_gateway", "terminate_gateway"):
            assert getattr(cls, m) is not getattr(Compute, m), f"{bt.value} advertises gateways without {m}"
    for bt in BACKENDS_WITH_VOLUMES_SUPPORT:
        cls = cls_of(bt)
        for m in ("create_volume", "delete_volume", "register_volume"):
            assert getattr(cls, m) is not getattr(Compute, m), f"{bt.value} advertises volumes without {m}"


def test_bootstrap_scripts_quote_ssh_keys(tmp_path):
    """Keys whose comments hold quotes, colons or '#' survive cloud-init YAML and the container
    bootstrap's shell (reference: compute.py get_user_data / get_docker_commands)."""
    import subprocess

    import yaml

    from dstack_amd.core.backends.base import get_docker_commands, get_user_data

    keys = ["ssh-ed25519 AAAAone alice's laptop", "ssh-rsa AAAAtwo build: #42 $(touch pwned)"]
    doc = yaml.safe_load(get_user_data(keys, "https://x/shim", "https://x/runner"))
    assert doc["ssh_authorized_keys"] == keys
    cmds = get_docker_commands(keys, "https://x/runner")
    step = next(c for c in cmds if "authorized_keys" in c and "printf" in c)
    home = tmp_path / "home"
    (home / ".ssh").mkdir(parents=True)
    r = subprocess.run(["sh", "-c", step], env={"HOME": str(home), "PATH": "/usr/bin:/bin"}, cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert (home / ".ssh" / "authorized_keys").read_text() == "".join(k + "\n" for k in keys)
    assert not (tmp_path / "pwned").exists()


@pytest.mark.parametrize("public", [True, False])
def test_aws_gateway_public_and_private(public):
    """AWS gateways: public in the default VPC; ``public_ip: false`` goes into the named VPC's
    subnet with no public address and is served on its private IP (reference: AWS is the backend
    with private gateways)."""
    from dstack_amd.core.models.gateways import GatewayComputeConfiguration

    calls = []

    def handler(req):
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        calls.append(form)
        a = form["Action"]
        if a == "DescribeImages":
            return _ec2x("<imagesSet><item><imageId>ami-1</imageId><creationDate>2024</creationDate></item></imagesSet>")
        if a == "DescribeSecurityGroups":
            return _ec2x("<securityGroupInfo><item><groupId>sg-gw</groupId></item></securityGroupInfo>")
        if a == "AuthorizeSecurityGroupIngress":
            return _ec2x("<return>true</return>")
        if a == "DescribeVpcs":
            return _ec2x("<vpcSet><item><vpcId>vpc-9</vpcId></item></vpcSet>")
        if a == "DescribeSubnets":
            return _ec2x("<subnetSet><item><subnetId>subnet-priv</subnetId><availabilityZone>us-east-1a"
                         "</availabilityZone><mapPublicIpOnLaunch>false</mapPublicIpOnLaunch></item></subnetSet>")
        if a == "RunInstances":
            return _ec2x("<instancesSet><item><instanceId>i-gw</instanceId></item></instancesSet>")
        if a == "DescribeInstances":
            return _ec2x("<reservationSet><item><instancesSet><item><instanceState><name>running</name></instanceState>"
                         "<ipAddress>54.1.1.1</ipAddress><privateIpAddress>10.0.3.7</privateIpAddress>"
                         "</item></instancesSet></item></reservationSet>")
        return httpx.Response(400, text="<Response><Errors><Error><Code>X</Code></Error></Errors></Response>")

    config = {} if public else {"vpc_name": "inner"}
    c = compute_class(BackendType.AWS)(config, {"access_key": "a", "secret_key": "s"}, _client(handler))
    conf = GatewayComputeConfiguration(project_name="main", instance_name="gw-1", backend=BackendType.AWS,
                                       region="us-east-1", public_ip=public, ssh_key_pub="ssh-rsa AAA gw")
    gpd = c.create_gateway(conf)
    run = next(x for x in calls if x["Action"] == "RunInstances")
    if public:
        assert gpd.ip_address == "54.1.1.1" and run["SecurityGroupId.1"] == "sg-gw"
    else:
        assert gpd.ip_address == "10.0.3.7"
        assert run["NetworkInterface.1.SubnetId"] == "subnet-priv"
        assert run["NetworkInterface.1.AssociatePublicIpAddress"] == "false"


def _ec2x(body):
    return httpx.Response(200, text=f'<R xmlns="http://ec2.amazonaws.com/doc/2016-11-15/">{body}</R>')


def test_cudo_start_script_is_shell_and_capacity_errors_map():
    bodies, state = [], {"code": None}

    def handler(req):
        if req.method == "POST" and req.url.path.endswith("/vm"):
            if state["code"] is not None:
                return httpx.Response(400, json={"code": state["code"], "message": "m"})
            bodies.append(json.loads(req.content))
            return httpx.Response(200, json={"id": "x"})
        if "/vms/" in req.url.path and req.method == "GET":
            return httpx.Response(200, json={"VM": {"state": "ACTIVE", "externalIpAddress": "5.5.5.5",
                                                   "internalIpAddress": "10.0.0.5"}})
        return httpx.Response(200, json={})

    c = compute_class(BackendType.CUDO)({"project_id": "p"}, {"api_key": "k"}, _client(handler))
    offer = _offer(c, "MI300X:4")
    jpd = c.create_instance(offer, CFG)
    b = bodies[0]
    assert b["startScript"].startswith("#!/bin/bash\n") and "#cloud-config" not in b["startScript"]
    assert "dstack-shim" in b["startScript"] and b["vmId"] == f"run-0-0-{offer.region}"[:60]
    assert b["customSshKeys"] == [CFG.ssh_keys[0].public]
    assert b["bootDiskImageId"] == "ubuntu-2204"  # AMD GPUs: not the NVIDIA driver image
    c.update_provisioning_data(jpd)
    assert (jpd.hostname, jpd.internal_ip) == ("5.5.5.5", "10.0.0.5")
    state["code"] = 3
    with pytest.raises(NoCapacityError):
        c.create_instance(offer, CFG)
    state["code"] = 9
    from dstack_amd.core.errors import ComputeError

    with pytest.raises(ComputeError, match="cudo create"):
        c.create_instance(offer, CFG)


def test_cloud_init_installs_the_amd_driver_only_when_missing(tmp_path):
    """The bootstrap installs amdgpu (DKMS) before the shim when the host has an Instinct GPU but no
    /dev/kfd; on CPU hosts (or with the driver present) the step does nothing and succeeds."""
    from dstack_amd.core.backends.base import get_amd_driver_commands, get_user_data

    ud = get_user_data(["ssh-ed25519 AAAA k"], "https://x/shim", "https://x/runner")
    lines = [json.loads(line[4:]) for line in ud.splitlines() if line.startswith("  - ") and "amdgpu" in line]
    assert len(lines) == 1 and "amdgpu-install -y --usecase=dkms" in lines[0]
    assert ud.index("amdgpu-install") < ud.index("dstack-shim")  # driver first, then the shim
    # run the step with stand-in tools: lspci reports no AMD GPU -> nothing installed, exit 0
    bin_dir = tmp_path / "bin"
    bin_dir.mkdir()
    (bin_dir / "lspci").write_text("#!/bin/sh\necho '00:02.0 VGA compatible controller [0300]: Intel [8086:46a6]'\n")
    (bin_dir / "curl").write_text(f"#!/bin/sh\ntouch {tmp_path}/curl-called\nexit 1\n")
    for f in bin_dir.iterdir():
        f.chmod(0o755)
    marker, log = tmp_path / "failed", tmp_path / "log"
    (tmp_path / "os-release").write_text('NAME="Ubuntu"\nVERSION_CODENAME=noble\n')
    script = get_amd_driver_commands(marker=str(marker), log=str(log), os_release=str(tmp_path / "os-release"))[0]
    # stand-ins for every tool the installer path calls: no network, no real package manager
    (bin_dir / "curl").write_text(f"#!/bin/sh\necho \"$@\" >> {tmp_path}/curl-called\nexit 1\n")
    (bin_dir / "apt-get").write_text(f"#!/bin/sh\necho \"$@\" >> {tmp_path}/apt-called\n")
    (bin_dir / "uname").write_text("#!/bin/sh\necho 6.8.0-1-test\n")
    (bin_dir / "modprobe").write_text("#!/bin/sh\nexit 1\n")
    for f in bin_dir.iterdir():
        f.chmod(0o755)
    env = {"PATH": f"{bin_dir}:/usr/bin:/bin"}
    assert subprocess.run(["bash", "-c", script], env=env).returncode == 0
    assert not (tmp_path / "curl-called").exists() and not marker.exists()
    if os.path.exists("/dev/kfd"):
        return  # a GPU box with the driver loaded: the installer path never runs
    # an MI355X (1002:75a3) without /dev/kfd: the ROCm 7 driver for this Ubuntu's codename, kernel
    # headers first; the (stand-in) download fails, so the marker carries the reason
    (bin_dir / "lspci").write_text("#!/bin/sh\necho '05:00.0 Processing accelerators [1200]: AMD [1002:75a3]'\n")
    subprocess.run(["bash", "-c", script], env=env)
    url = (tmp_path / "curl-called").read_text()
    assert "amdgpu-install/7.0/ubuntu/noble/amdgpu-install_7.0." in url, url
    assert "linux-headers-6.8.0-1-test" in (tmp_path / "apt-called").read_text()
    text = marker.read_text()
    assert "amdgpu 7.0 driver install failed on ubuntu/noble kernel 6.8.0-1-test: /dev/kfd missing" in text
    # an MI210 (1002:740f): the 6.4 driver
    (tmp_path / "curl-called").unlink()
    (bin_dir / "lspci").write_text("#!/bin/sh\necho '05:00.0 Processing accelerators [1200]: AMD [1002:740f]'\n")
    subprocess.run(["bash", "-c", script], env=env)
    assert "amdgpu-install/6.4/ubuntu/noble/amdgpu-install_6.4." in (tmp_path / "curl-called").read_text()
