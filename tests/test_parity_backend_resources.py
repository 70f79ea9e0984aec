"""Backend resource helpers, case by case against the reference's
``src/tests/_internal/core/backends/{aws,azure,gcp,kubernetes,oci}/test_*.py``: cloud tag/label rules
(and their use in configs and launches), OS image choice, Kubernetes GPU discovery from node labels,
OCI shape quotas and security-rule comparison.  Clouds are ``httpx.MockTransport`` fakes."""

from __future__ import annotations

import urllib.parse

import httpx
import pytest

from dstack_amd.core.backends.clouds import tags as T
from dstack_amd.core.errors import BackendError, ComputeResourceNotFoundError


# ---- aws/test_resources.py: tags ------------------------------------------------------------------
@pytest.mark.parametrize("key", ["Environment", "Project123", "special-chars-+/@=:_", "a" * 128])
def test_aws_valid_tag_key(key):
    assert T.aws_tag_key_ok(key)


@pytest.mark.parametrize("key", ["aws:reserved", "key\twith\nweird\nspaces", "", "a" * 129, "Invalid#Char"])
def test_aws_invalid_tag_key(key):
    assert not T.aws_tag_key_ok(key)


@pytest.mark.parametrize("value", ["Production", "v1.0", "", "a" * 256])
def test_aws_valid_tag_value(value):
    assert T.aws_tag_value_ok(value)


@pytest.mark.parametrize("value", ["a" * 257, "Invalid#Value"])
def test_aws_invalid_tag_value(value):
    assert not T.aws_tag_value_ok(value)


def test_aws_validate_tags():
    assert T.validate_tags("aws", {"Environment": "Production", "Project": "AWS_Tag_Validator"}) is None
    with pytest.raises(BackendError, match="Invalid resource tags") as ei:
        T.validate_tags("aws", {"aws:ReservedKey": "SomeValue", "ValidKey": "Invalid#Value"})
    assert "'aws:ReservedKey'" in str(ei.value) and "'ValidKey'" in str(ei.value)


# ---- azure/test_resources.py -------------------------------------------------------------------------
@pytest.mark.parametrize("key", ["Environment", "Project123", "key with spaces", "a" * 512, "ключ"])
def test_azure_valid_tag_keys(key):
    assert T.azure_tag_key_ok(key)


@pytest.mark.parametrize("key", ["", "a" * 513, "key<", "key>", "key&", "key\\", "key%", "key?", "key/"])
def test_azure_invalid_tag_keys(key):
    assert not T.azure_tag_key_ok(key)


@pytest.mark.parametrize("value", ["", "Production", "v1.0 <any> & chars/%?", "a" * 256])
def test_azure_valid_tag_values(value):
    assert T.azure_tag_value_ok(value)


def test_azure_invalid_tag_values_and_validate():
    assert not T.azure_tag_value_ok("a" * 257)
    assert T.validate_tags("azure", {"Environment": "Production", "Team": "R&D / ML"}) is None
    with pytest.raises(BackendError, match="Invalid Azure resource tags"):
        T.validate_tags("azure", {"bad/key": "v"})


# ---- gcp/test_resources.py ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["a", "dstack-project", "with_underscore", "a" * 63, "x1-2_3"])
def test_gcp_valid_resource_name(name):
    assert T.gcp_resource_name_ok(name)


@pytest.mark.parametrize("name", ["", "1starts-with-digit", "-dash", "Upper", "a" * 64, "dot.name", "space name"])
def test_gcp_invalid_resource_name(name):
    assert not T.gcp_resource_name_ok(name)


@pytest.mark.parametrize("value,ok", [("", True), ("1digit-first", True), ("a" * 63, True), ("a" * 64, False),
                                      ("UPPER", False), ("with.dot", False)])
def test_gcp_label_value(value, ok):
    assert T.gcp_label_value_ok(value) is ok


def test_gcp_validate_labels():
    assert T.validate_tags("gcp", {"env": "prod", "team": "ml-infra"}) is None
    with pytest.raises(BackendError, match="Invalid resource labels"):
        T.validate_tags("gcp", {"Env": "prod"})
    with pytest.raises(BackendError, match="Invalid resource labels"):
        T.validate_tags("gcp", {"env": "Prod"})


def test_backend_configs_reject_invalid_tags():
    """Configs are checked when a backend is configured (API or server config.yml)."""
    from pydantic import ValidationError

    from dstack_amd.core.models.backend_configs import AWSConfig, AzureConfig, GCPConfig

    assert AWSConfig(tags={"team": "ml"}).tags == {"team": "ml"}
    with pytest.raises(ValidationError, match="Invalid resource tags"):
        AWSConfig(tags={"aws:x": "y"})
    with pytest.raises(ValidationError, match="Invalid Azure resource tags"):
        AzureConfig(tenant_id="t", subscription_id="s", tags={"a/b": "c"})
    with pytest.raises(ValidationError, match="Invalid resource labels"):
        GCPConfig(project_id="p", tags={"Team": "ml"})


def test_merged_tags_keep_dstack_ownership_keys():
    assert T.merged_tags("aws", {"owner": "dstack", "Name": "i"}, {"tags": {"owner": "me", "team": "ml"}}) == \
        {"owner": "dstack", "Name": "i", "team": "ml"}


# ---- aws/test_resources.py: images ------------------------------------------------------------------
def _xml(body):
    return f'<R xmlns="http://ec2.amazonaws.com/doc/2016-11-15/">{body}</R>'


def _aws(images, config=None, calls=None):
    from dstack_amd.core.backends.clouds.aws import AWSCompute

    def handler(req):
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        if calls is not None:
            calls.append(form)
        items = "".join(f"<item><imageId>{i}</imageId><imageState>{st}</imageState><creationDate>{d}</creationDate>"
                        "</item>" for i, st, d in images)
        return httpx.Response(200, text=_xml(f"<imagesSet>{items}</imagesSet>"))

    return AWSCompute(config or {}, {"access_key": "AK", "secret_key": "SK"},
                      httpx.Client(transport=httpx.MockTransport(handler)))


def test_aws_image_returns_the_latest_available():
    c = _aws([("ami-1", "failed", "2024-01-01T00:00:00.000Z"), ("ami-2", "available", "2022-01-01T00:00:00.000Z"),
              ("ami-3", "available", "2023-01-01T00:00:00.000Z")])
    assert c.image_id_and_username("us-east-1", gpu=False) == ("ami-3", "ubuntu")


def test_aws_image_raises_resource_not_found_if_none_available(caplog):
    c = _aws([("ami-1", "failed", "2000-01-01T00:00:00.000Z")])
    with pytest.raises(ComputeResourceNotFoundError):
        c.image_id_and_username("us-east-1", gpu=False)
    assert "ubuntu-jammy-22.04" in caplog.text and "not found" in caplog.text


@pytest.mark.parametrize("gpu", [False, True])
def test_aws_image_default_is_canonical_ubuntu(gpu):
    calls = []
    c = _aws([("ami-1", "available", "2024-01-01")], calls=calls)
    assert c.image_id_and_username("us-east-1", gpu) == ("ami-1", "ubuntu")
    assert calls[0]["Owner.1"] == "099720109477" and calls[0]["Filter.1.Value.1"].startswith("ubuntu/images/")


@pytest.mark.parametrize("gpu,name,owner,user", [(False, "cpu-ami", "123456789012", "debian"),
                                                 (True, "rocm-ami", "self", "dstack")])
def test_aws_image_uses_image_config_if_provided(gpu, name, owner, user):
    calls = []
    cfg = {"os_images": {"cpu": {"name": "cpu-ami", "owner": "123456789012", "user": "debian"},
                         "amd": {"name": "rocm-ami", "user": "dstack"}}}
    c = _aws([("ami-9", "available", "2024-01-01")], cfg, calls)
    assert c.image_id_and_username("us-east-1", gpu) == ("ami-9", user)
    assert (calls[0]["Filter.1.Value.1"], calls[0]["Owner.1"]) == (name, owner)


def test_aws_image_raises_if_image_config_kind_not_set(caplog):
    c = _aws([("ami-9", "available", "2024-01-01")], {"os_images": {"amd": {"name": "rocm-ami"}}})
    with pytest.raises(ComputeResourceNotFoundError):
        c.image_id_and_username("us-east-1", gpu=False)
    assert "cpu image not configured" in caplog.text


def test_aws_launch_uses_configured_image_user_and_tags():
    from dstack_amd.core.backends.base import offer_matches  # noqa: F401  (catalog import side effects)
    from dstack_amd.core.backends.clouds.aws import AWSCompute
    from dstack_amd.core.models.instances import InstanceConfiguration, SSHKey
    from dstack_amd.core.models.resources import ResourcesSpec
    from dstack_amd.core.models.runs import Requirements

    calls = []

    def handler(req):
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        calls.append(form)
        a = form["Action"]
        if a == "DescribeImages":
            return httpx.Response(200, text=_xml("<imagesSet><item><imageId>ami-r</imageId><imageState>available"
                                                 "</imageState><creationDate>2025</creationDate></item></imagesSet>"))
        if a == "DescribeSecurityGroups":
            return httpx.Response(200, text=_xml("<securityGroupInfo><item><groupId>sg-1</groupId></item>"
                                                 "</securityGroupInfo>"))
        if a == "RunInstances":
            return httpx.Response(200, text=_xml("<instancesSet><item><instanceId>i-1</instanceId></item>"
                                                 "</instancesSet>"))
        return httpx.Response(200, text=_xml(""))

    c = AWSCompute({"os_images": {"amd": {"name": "rocm-ami", "user": "rocm"}, "cpu": {"name": "c", "user": "debian"}},
                    "tags": {"team": "ml", "owner": "someone-else"}},
                   {"access_key": "AK", "secret_key": "SK"}, httpx.Client(transport=httpx.MockTransport(handler)))
    offer = c.get_offers(Requirements(resources=ResourcesSpec.model_validate({"gpu": 0})))[0]
    jpd = c.create_instance(offer, InstanceConfiguration(project_name="main", instance_name="i", user="u",
                                                         ssh_keys=[SSHKey(public="ssh-ed25519 AAAA")]))
    assert jpd.username == "debian"
    run = next(f for f in calls if f["Action"] == "RunInstances")
    assert run["ImageId"] == "ami-r"
    tags = {run[f"TagSpecification.1.Tag.{i}.Key"]: run[f"TagSpecification.1.Tag.{i}.Value"]
            for i in range(1, 10) if f"TagSpecification.1.Tag.{i}.Key" in run}
    assert tags["team"] == "ml" and tags["owner"] == "dstack" and tags["dstack_project"] == "main"


# ---- azure/test_compute.py ----------------------------------------------------------------------------
def _itype(name, gpus, vendor=None):
    from dstack_amd.core.models.instances import Gpu, InstanceType, Resources

    return InstanceType(name=name, resources=Resources(
        cpus=6, memory_mib=55000, spot=True, gpus=[Gpu(name=g, memory_mib=16000, vendor=vendor) for g in gpus]))


@pytest.mark.parametrize("itype,variant", [
    (_itype("Standard_ND96isr_MI300X_v5", ["MI300X"] * 8, "amd"), "ROCM"),
    (_itype("Standard_NV6ads_A10_v5", ["A10"], "nvidia"), "NVIDIA"),
    (_itype("Standard_NC4as_T4_v3", ["T4"]), "NVIDIA"),
    (_itype("Standard_DS1_v2", []), "STANDARD"),
])
def test_azure_image_variant_from_instance_type(itype, variant):
    from dstack_amd.core.backends.clouds.hyperscalers import AzureImageVariant

    assert AzureImageVariant.from_instance_type(itype) is AzureImageVariant[variant]


def test_azure_image_reference_and_override():
    from dstack_amd.core.backends.clouds.hyperscalers import AzureImageVariant as V

    assert V.ROCM.image_reference()["sku"] == "2204-rocm"
    assert V.STANDARD.image_reference()["publisher"] == "Canonical"
    over = {"rocm": {"publisher": "me", "offer": "img", "sku": "1"}}
    assert V.ROCM.image_reference(over) == {"publisher": "me", "offer": "img", "sku": "1", "version": "latest"}
    assert V.STANDARD.image_reference(over)["publisher"] == "Canonical"


def test_azure_template_tags_every_resource():
    from dstack_amd.core.backends.clouds.hyperscalers import AzureCompute, AzureImageVariant

    c = AzureCompute.__new__(AzureCompute)
    c.config = {"tags": {"team": "ml"}}
    tpl = c._template("vm", "Standard_ND96isr_MI300X_v5", "eastus", "#cloud-config", 100, False, ["ssh-ed25519 A"],
                      image=AzureImageVariant.ROCM.image_reference(), tags={"dstack_project": "main"})
    assert all(r["tags"] == {"team": "ml", "owner": "dstack", "dstack_project": "main"} for r in tpl["resources"])
    vm = next(r for r in tpl["resources"] if r["type"] == "Microsoft.Compute/virtualMachines")
    assert vm["properties"]["storageProfile"]["imageReference"]["sku"] == "2204-rocm"


# ---- kubernetes/test_compute.py -----------------------------------------------------------------------
def test_k8s_no_gpus_if_no_labels():
    from dstack_amd.core.backends.clouds.containers import gpus_from_node_labels

    assert gpus_from_node_labels({}) == []


def test_k8s_no_gpus_if_missing_labels():
    from dstack_amd.core.backends.clouds.containers import gpus_from_node_labels

    assert gpus_from_node_labels({"nvidia.com/gpu.count": 1}) == []
    assert gpus_from_node_labels({}, {"amd.com/gpu": "8"}) == []  # AMD GPUs of an unknown model: not guessed


def test_k8s_correct_memory_for_different_gpus():
    from dstack_amd.core.backends.clouds.containers import gpus_from_node_labels

    g = gpus_from_node_labels({"nvidia.com/gpu.count": 1, "nvidia.com/gpu.product": "A100-SXM4-40GB"})
    assert [(x.name, x.memory_mib) for x in g] == [("A100", 40 * 1024)]
    g = gpus_from_node_labels({"nvidia.com/gpu.count": 1, "nvidia.com/gpu.product": "A100-SXM4-80GB"})
    assert [(x.name, x.memory_mib) for x in g] == [("A100", 80 * 1024)]
    g = gpus_from_node_labels({"amd.com/gpu.product-name": "AMD_Instinct_MI300X_OAM", "amd.com/gpu.vram": "192G"},
                              {"amd.com/gpu": "8"})
    assert [(x.name, x.memory_mib, x.vendor.value) for x in g] == [("MI300X", 192 * 1024, "amd")] * 8
    g = gpus_from_node_labels({"amd.com/gpu.device-id": "75a3"}, {"amd.com/gpu": "2"})
    assert [(x.name, x.memory_mib) for x in g] == [("MI355X", 288 * 1024)] * 2  # memory from the catalog


# ---- oci/test_resources.py -----------------------------------------------------------------------------
def _quota():
    from dstack_amd.core.backends.clouds.hyperscalers import ShapesQuota

    return ShapesQuota({"region-1": {"region-1-ad-1": {"shape.1", "shape.2"}, "region-1-ad-2": {"shape.2", "shape.3"}},
                        "region-2": {"region-2-ad-1": {"shape.1", "shape.3"}}})


@pytest.mark.parametrize("shape,region,ok", [
    ("shape.1", "region-1", True), ("shape.2", "region-1", True), ("shape.3", "region-1", True),
    ("shape.1", "region-2", True), ("shape.2", "region-2", False), ("shape.3", "region-2", True),
    ("shape.9", "region-1", False), ("shape.1", "region-9", False)])
def test_oci_is_within_region_quota(shape, region, ok):
    assert _quota().is_within_region_quota(shape, region) is ok


@pytest.mark.parametrize("shape,ad,ok", [
    ("shape.1", "region-1-ad-1", True), ("shape.3", "region-1-ad-1", False), ("shape.1", "region-1-ad-2", False),
    ("shape.3", "region-1-ad-2", True), ("shape.1", "region-2-ad-1", True), ("shape.2", "region-2-ad-1", False),
    ("shape.9", "region-1-ad1", False), ("shape.1", "region-9-ad-9", False)])
def test_oci_is_within_domain_quota(shape, ad, ok):
    assert _quota().is_within_domain_quota(shape, ad) is ok
    assert _quota().domains_for("shape.2", "region-1") == ["region-1-ad-1", "region-1-ad-2"]


def test_oci_security_rules_equal_after_conversion():
    from dstack_amd.core.backends.clouds.hyperscalers import SecurityRule

    api = {"protocol": "all", "source": "0.0.0.0/0", "sourceType": "CIDR_BLOCK", "isStateless": False,
           "id": "AAAAAA", "timeCreated": "2024-05-01T10:00:00Z", "description": None}
    assert SecurityRule("INGRESS", "all", "0.0.0.0/0") == SecurityRule.from_api(api, "INGRESS")
    r = SecurityRule("INGRESS", "6", "0.0.0.0/0", ports=(22, 22))
    assert SecurityRule.from_api(r.to_api(), "INGRESS") == r


def test_oci_security_rules_unequal_after_conversion():
    from dstack_amd.core.backends.clouds.hyperscalers import SecurityRule

    api = {"protocol": "all", "source": "10.10.10.0/24", "sourceType": "CIDR_BLOCK", "isStateless": False,
           "id": "AAAAAA"}
    assert SecurityRule("INGRESS", "all", "0.0.0.0/0") != SecurityRule.from_api(api, "INGRESS")
    assert SecurityRule("EGRESS", "all", "10.10.10.0/24") != SecurityRule.from_api(api, "INGRESS")
