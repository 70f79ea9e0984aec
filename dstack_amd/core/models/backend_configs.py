"""Per-backend configuration contract: what ``projects[].backends[]`` in the server's ``config.yml``
and the ``/api/project/{p}/backends/create|update(_yaml)`` endpoints accept (reference:
``C/models/backends/{aws,azure,gcp,oci,lambdalabs,vultr,tensordock,cudo,datacrunch,nebius,runpod,
vastai,kubernetes}.py`` — the same YAML keys and credential types, so a reference server config
loads unchanged).

Every backend is one model discriminated by ``type``; credentials are a nested union discriminated
by ``creds.type``.  ``split_backend_config`` validates a raw mapping and returns (config without
secrets, secrets) — the server stores the two in separate columns, the secrets encrypted, and never
returns the secrets from ``config_info``/``get_yaml``.
"""

from __future__ import annotations

from typing import Annotated, Dict, List, Literal, Optional, Tuple, Union

from pydantic import Field, ValidationError, field_validator

from dstack_amd.core.errors import ServerClientError
from dstack_amd.core.models.common import CoreModel


class _Input(CoreModel):
    model_config = {"extra": "forbid"}


# ---- credential types -----------------------------------------------------------------------------
class AccessKeyCreds(_Input):
    type: Literal["access_key"] = "access_key"
    access_key: str
    secret_key: str
    session_token: Optional[str] = None


class DefaultCreds(_Input):
    """Use the environment's credentials (instance role, CLI config, env vars)."""

    type: Literal["default"] = "default"


class ClientCreds(_Input):  # Azure service principal
    type: Literal["client"] = "client"
    client_id: str
    client_secret: str
    tenant_id: Optional[str] = None


class ServiceAccountCreds(_Input):  # GCP / Nebius service-account key file (contents in ``data``)
    type: Literal["service_account"] = "service_account"
    filename: Optional[str] = None
    data: str


class OCIClientCreds(_Input):
    type: Literal["client"] = "client"
    user: str
    tenancy: str
    key_file: Optional[str] = None
    key_content: Optional[str] = None
    pass_phrase: Optional[str] = None
    fingerprint: str
    region: str


class OCIDefaultCreds(_Input):
    type: Literal["default"] = "default"
    file: str = "~/.oci/config"
    profile: str = "DEFAULT"


class APIKeyCreds(_Input):
    type: Literal["api_key"] = "api_key"
    api_key: str


class TensorDockCreds(_Input):
    type: Literal["api_key"] = "api_key"
    api_key: str
    api_token: str


class DataCrunchCreds(_Input):
    type: Literal["api_key"] = "api_key"
    client_id: str
    client_secret: str


class IAMTokenCreds(_Input):
    """A pre-issued Nebius IAM token (addition to the reference's service-account creds)."""

    type: Literal["iam_token"] = "iam_token"
    iam_token: str


# ---- backend configs ---------------------------------------------------------------------------
def _check_tags(cloud: str, tags: Optional[Dict[str, str]]) -> Optional[Dict[str, str]]:
    from dstack_amd.core.backends.clouds.tags import validate_tags
    from dstack_amd.core.errors import BackendError

    try:
        validate_tags(cloud, tags)
    except BackendError as e:
        raise ValueError(str(e)) from None
    return tags


class AWSOSImage(_Input):
    name: str
    owner: str = "self"
    user: str = "ubuntu"


class AWSOSImages(_Input):
    cpu: Optional[AWSOSImage] = None
    amd: Optional[AWSOSImage] = None  # ROCm image for AMD Instinct instances
    nvidia: Optional[AWSOSImage] = None


class AWSConfig(_Input):
    type: Literal["aws"] = "aws"
    regions: Optional[List[str]] = None
    vpc_name: Optional[str] = None
    vpc_ids: Optional[Dict[str, str]] = None
    subnet_ids: Optional[Dict[str, str]] = None
    default_vpcs: Optional[bool] = None
    public_ips: Optional[bool] = None
    tags: Optional[Dict[str, str]] = None
    os_images: Optional[AWSOSImages] = None
    creds: Annotated[Union[AccessKeyCreds, DefaultCreds], Field(discriminator="type")] = DefaultCreds()

    @field_validator("tags")
    @classmethod
    def _valid_tags(cls, v):
        return _check_tags("aws", v)


class AzureConfig(_Input):
    type: Literal["azure"] = "azure"
    tenant_id: str
    subscription_id: str
    locations: Optional[List[str]] = None
    regions: Optional[List[str]] = None
    vpc_ids: Optional[Dict[str, str]] = None
    resource_groups: Optional[Dict[str, str]] = None
    subnet_id: Optional[str] = None
    public_ips: Optional[bool] = None
    tags: Optional[Dict[str, str]] = None
    vm_images: Optional[Dict[str, Dict[str, str]]] = None  # AzureImageVariant overrides: rocm/nvidia/standard
    creds: Annotated[Union[ClientCreds, DefaultCreds], Field(discriminator="type")] = DefaultCreds()

    @field_validator("tags")
    @classmethod
    def _valid_tags(cls, v):
        return _check_tags("azure", v)


class GCPConfig(_Input):
    type: Literal["gcp"] = "gcp"
    project_id: str
    regions: Optional[List[str]] = None
    zones: Optional[Dict[str, str]] = None
    vpc_name: Optional[str] = None
    vpc_project_id: Optional[str] = None
    public_ips: Optional[bool] = None
    nat_check: Optional[bool] = None
    vm_service_account: Optional[str] = None
    tags: Optional[Dict[str, str]] = None
    creds: Annotated[Union[ServiceAccountCreds, DefaultCreds], Field(discriminator="type")] = DefaultCreds()

    @field_validator("tags")
    @classmethod
    def _valid_tags(cls, v):
        return _check_tags("gcp", v)


class OCIConfig(_Input):
    type: Literal["oci"] = "oci"
    regions: Optional[List[str]] = None
    compartment_id: Optional[str] = None
    subnet_ids: Optional[Dict[str, str]] = None
    images: Optional[Dict[str, str]] = None
    availability_domains: Optional[Dict[str, str]] = None
    creds: Annotated[Union[OCIClientCreds, OCIDefaultCreds], Field(discriminator="type")] = OCIDefaultCreds()


class LambdaConfig(_Input):
    type: Literal["lambda"] = "lambda"
    regions: Optional[List[str]] = None
    creds: APIKeyCreds


class VultrConfig(_Input):
    type: Literal["vultr"] = "vultr"
    regions: Optional[List[str]] = None
    images: Optional[Dict[str, str]] = None  # {"instance" | "bare_metal": os id or marketplace image id}
    creds: APIKeyCreds


class TensorDockConfig(_Input):
    type: Literal["tensordock"] = "tensordock"
    regions: Optional[List[str]] = None
    creds: TensorDockCreds


class CudoConfig(_Input):
    type: Literal["cudo"] = "cudo"
    project_id: str
    regions: Optional[List[str]] = None
    images: Optional[Dict[str, str]] = None  # boot image id by kind: amd / nvidia / cpu
    creds: APIKeyCreds


class DataCrunchConfig(_Input):
    type: Literal["datacrunch"] = "datacrunch"
    regions: Optional[List[str]] = None
    creds: DataCrunchCreds


class NebiusConfig(_Input):
    type: Literal["nebius"] = "nebius"
    cloud_id: Optional[str] = None
    folder_id: str
    network_id: Optional[str] = None
    subnet_id: Optional[str] = None
    image_id: Optional[str] = None
    regions: Optional[List[str]] = None
    creds: Annotated[Union[ServiceAccountCreds, IAMTokenCreds], Field(discriminator="type")]


class RunpodConfig(_Input):
    type: Literal["runpod"] = "runpod"
    regions: Optional[List[str]] = None
    creds: APIKeyCreds


class VastAIConfig(_Input):
    type: Literal["vastai"] = "vastai"
    regions: Optional[List[str]] = None
    creds: APIKeyCreds


class KubernetesNetworking(_Input):
    ssh_host: Optional[str] = None
    ssh_port: Optional[int] = None


class Kubeconfig(_Input):
    filename: Optional[str] = None
    data: str


class KubernetesConfig(_Input):
    type: Literal["kubernetes"] = "kubernetes"
    namespace: Optional[str] = None
    api_url: Optional[str] = None
    networking: KubernetesNetworking = KubernetesNetworking()
    kubeconfig: Kubeconfig  # the cluster credentials (stored with the secrets)


class DstackConfig(_Input):
    type: Literal["dstack"] = "dstack"
    base_backends: List[str] = []


AnyBackendConfig = Annotated[
    Union[AWSConfig, AzureConfig, GCPConfig, OCIConfig, LambdaConfig, VultrConfig, TensorDockConfig, CudoConfig,
          DataCrunchConfig, NebiusConfig, RunpodConfig, VastAIConfig, KubernetesConfig, DstackConfig],
    Field(discriminator="type"),
]


class _Wrapper(CoreModel):
    config: AnyBackendConfig


# secret-bearing keys per backend type (everything else is plain configuration)
_SECRET_KEYS = {"kubernetes": ("kubeconfig",)}


def parse_backend_config(raw: dict):
    """Validate a backend mapping; a bad one raises ``ServerClientError`` naming the fields."""
    if not isinstance(raw, dict) or "type" not in raw:
        raise ServerClientError("Backend config must be a mapping with a 'type'")
    try:
        return _Wrapper.model_validate({"config": raw}).config
    except ValidationError as e:
        errs = "; ".join(f"{'.'.join(str(x) for x in err['loc'][2:]) or 'config'}: {err['msg']}"
                         for err in e.errors())
        raise ServerClientError(f"Invalid {raw.get('type')} backend config: {errs}") from None


def split_backend_config(raw: dict) -> Tuple[str, dict, dict]:
    """(type, config without secrets, secrets) of a validated backend mapping."""
    model = parse_backend_config(raw)
    data = model.model_dump(mode="json", exclude_none=True)
    btype = data.pop("type")
    secret_keys = _SECRET_KEYS.get(btype, ("creds",))
    secrets = {}
    for k in secret_keys:
        if k in data:
            v = data.pop(k)
            if k == "creds":
                secrets.update(v)
            else:
                secrets[k] = v
    return btype, data, secrets


# ---- form descriptors for the web UI ------------------------------------------------------------
def _describe(name: str, annotation, required: bool) -> dict:
    """A small, UI-friendly description of one config field (the JSON schema's $ref/anyOf forms are
    more than a form renderer needs): str | int | bool | list | map | object | union."""
    import typing

    origin, args = typing.get_origin(annotation), typing.get_args(annotation)
    if origin is typing.Annotated:
        return _describe(name, args[0], required)
    if origin is Union and type(None) in args:
        rest = [a for a in args if a is not type(None)]
        return _describe(name, rest[0] if len(rest) == 1 else Union[tuple(rest)], False)
    if origin is Union:
        variants = []
        for a in args:
            tf = a.model_fields["type"]
            variants.append({"type": tf.default, "fields": _model_fields(a)})
        return {"name": name, "kind": "union", "required": required, "variants": variants}
    if origin in (list, List):
        return {"name": name, "kind": "list", "required": required}
    if origin in (dict, Dict):
        return {"name": name, "kind": "map", "required": required}
    if isinstance(annotation, type) and issubclass(annotation, CoreModel):
        return {"name": name, "kind": "object", "required": required, "fields": _model_fields(annotation)}
    kind = {bool: "bool", int: "int", float: "float"}.get(annotation, "str")
    return {"name": name, "kind": kind, "required": required}


def _model_fields(cls) -> List[dict]:
    out = []
    for n, f in cls.model_fields.items():
        if n == "type":
            continue
        d = _describe(n, f.annotation, f.is_required())
        if f.description:
            d["help"] = f.description
        out.append(d)
    return out


def backend_form_schema() -> Dict[str, List[dict]]:
    """{backend type: [field descriptor]} for every configurable backend (web UI forms)."""
    import typing

    union = typing.get_args(typing.get_args(AnyBackendConfig)[0])
    return {cls.model_fields["type"].default: _model_fields(cls) for cls in union}
