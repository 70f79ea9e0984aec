"""The ``.dstack.yml`` contract: run/fleet/gateway/volume configurations, discriminated by ``type``
(reference: ``C/models/configurations.py:27-405``).  Accepts the reference's YAML verbatim."""

from __future__ import annotations

import re
from enum import Enum
from typing import Any, List, Literal, Optional, Union

from pydantic import Field, TypeAdapter, ValidationError, field_validator, model_validator
from typing_extensions import Annotated

from dstack_amd.core.errors import ConfigurationError
from dstack_amd.core.models.common import CoreModel, RegistryAuth
from dstack_amd.core.models.envs import Env
from dstack_amd.core.models.fleets import FleetConfiguration
from dstack_amd.core.models.gateways import GatewayConfiguration
from dstack_amd.core.models.profiles import ProfileParams
from dstack_amd.core.models.resources import IntRange, ResourcesSpec
from dstack_amd.core.models.services import AnyModel, OpenAIChatModel, ScalingSpec
from dstack_amd.core.models.unix import UnixUser
from dstack_amd.core.models.volumes import (
    InstanceMountPoint,
    MountPoint,
    VolumeConfiguration,
    VolumeMountPoint,
    parse_mount_point,
)

CommandsList = List[str]
SERVICE_HTTPS_DEFAULT = True
STRIP_PREFIX_DEFAULT = True


class RunConfigurationType(str, Enum):
    DEV_ENVIRONMENT = "dev-environment"
    TASK = "task"
    SERVICE = "service"


class PythonVersion(str, Enum):
    PY38 = "3.8"
    PY39 = "3.9"
    PY310 = "3.10"
    PY311 = "3.11"
    PY312 = "3.12"
    PY313 = "3.13"


def _valid_port(p: int) -> int:
    if not (0 < p <= 65536):
        raise ValueError(f"invalid port: {p}")
    return p


class PortMapping(CoreModel):
    local_port: Optional[int] = None
    container_port: int

    @classmethod
    def parse(cls, v: str) -> "PortMapping":
        """``8080`` | ``80:8080`` | ``*:8080``"""
        r = re.search(r"^(?:(\d+|\*):)?(\d+)?$", str(v))
        if not r or r.group(2) is None:
            raise ValueError(f"invalid port mapping: {v}")
        local, container = r.groups()
        if local is None:
            local_port = int(container)
        elif local == "*":
            local_port = None
        else:
            local_port = int(local)
        return cls(local_port=local_port, container_port=_valid_port(int(container)))


def _convert_port(v: Any) -> PortMapping:
    if isinstance(v, PortMapping):
        return v
    if isinstance(v, bool):
        raise ValueError(f"invalid port: {v}")
    if isinstance(v, int):
        _valid_port(v)
        return PortMapping(local_port=v, container_port=v)
    if isinstance(v, str):
        return PortMapping.parse(v)
    if isinstance(v, dict):
        return PortMapping.model_validate(v)
    raise ValueError(f"invalid port: {v!r}")


class BaseRunConfiguration(CoreModel):
    type: str
    name: Optional[str] = Field(None, description="Run name; random if omitted")
    image: Optional[str] = Field(None, description="Docker image (ROCm images for AMD GPUs)")
    user: Optional[str] = None
    privileged: bool = False
    entrypoint: Optional[str] = None
    working_dir: Optional[str] = None
    home_dir: str = "/root"  # deprecated, no effect
    registry_auth: Optional[RegistryAuth] = None
    python: Optional[PythonVersion] = None
    nvcc: Optional[bool] = None
    single_branch: Optional[bool] = None
    env: Env = Field(default_factory=Env)
    setup: CommandsList = []
    resources: ResourcesSpec = Field(default_factory=ResourcesSpec)
    volumes: List[Union[VolumeMountPoint, InstanceMountPoint]] = []

    @field_validator("python", mode="before")
    @classmethod
    def _python(cls, v, info):
        if v is not None and info.data.get("image"):
            raise ValueError("`image` and `python` are mutually exclusive fields")
        if isinstance(v, float):
            v = "3.10" if str(v) == "3.1" else str(v)
        return v

    @field_validator("volumes", mode="before")
    @classmethod
    def _volumes(cls, v):
        if v is None:
            return []
        return [parse_mount_point(x) for x in v]

    @field_validator("user")
    @classmethod
    def _user(cls, v):
        if v is not None:
            UnixUser.parse(v)
        return v


class _WithPorts(CoreModel):
    ports: List[PortMapping] = []

    @field_validator("ports", mode="before")
    @classmethod
    def _ports(cls, v):
        return [_convert_port(p) for p in (v or [])]


class _WithCommands(CoreModel):
    commands: CommandsList = []


class DevEnvironmentConfiguration(ProfileParams, _WithPorts, BaseRunConfiguration):
    type: Literal["dev-environment"] = "dev-environment"
    ide: Literal["vscode"]
    version: Optional[str] = Field(None, description="VS Code commit to pre-install the server of (Help > About)")
    init: CommandsList = []

    @field_validator("version")
    @classmethod
    def _commit(cls, v):
        import re

        if v is not None and not re.match(r"^[0-9a-f]{7,40}$", v):
            raise ValueError("version must be a VS Code commit hash (Help > About), e.g. 1a5daa3a0231a0fbba4f14db7ec463cf99d7768e")
        return v


class TaskConfiguration(ProfileParams, _WithCommands, _WithPorts, BaseRunConfiguration):
    type: Literal["task"] = "task"
    nodes: int = Field(1, ge=1, description="Number of nodes (one job per node)")

    @model_validator(mode="after")
    def _cmds(self):
        if not self.commands and not self.image:
            raise ValueError("Either `commands` or `image` must be set")
        return self


class ServiceConfiguration(ProfileParams, _WithCommands, BaseRunConfiguration):
    type: Literal["service"] = "service"
    port: PortMapping
    gateway: Optional[Union[bool, str]] = None
    strip_prefix: bool = STRIP_PREFIX_DEFAULT
    model: Optional[AnyModel] = None
    https: bool = SERVICE_HTTPS_DEFAULT
    auth: bool = True
    replicas: IntRange = Field(default_factory=lambda: IntRange(min=1, max=1))
    scaling: Optional[ScalingSpec] = None

    @field_validator("port", mode="before")
    @classmethod
    def _port(cls, v):
        if isinstance(v, int) and not isinstance(v, bool):
            return PortMapping(local_port=80, container_port=_valid_port(v))
        if isinstance(v, str):
            return PortMapping.parse(v)
        return v

    @field_validator("model", mode="before")
    @classmethod
    def _model(cls, v):
        if isinstance(v, str):
            return OpenAIChatModel(type="chat", name=v, format="openai")
        return v

    @field_validator("replicas", mode="before")
    @classmethod
    def _replicas(cls, v):
        if isinstance(v, str) and ".." in v:
            lo, hi = v.replace(" ", "").split("..", 1)
            v = IntRange(min=int(lo or 0), max=int(hi) if hi else None)
        elif isinstance(v, (int, float)) and not isinstance(v, bool):
            v = IntRange(min=int(v), max=int(v))
        elif isinstance(v, str):
            v = IntRange(min=int(v.strip()), max=int(v.strip()))
        elif isinstance(v, dict):
            v = IntRange(min=v.get("min", 0), max=v.get("max"))
        if v.max is None:
            raise ValueError("The maximum number of replicas is required")
        if (v.min or 0) < 0:
            raise ValueError("The minimum number of replicas must be greater than or equal to 0")
        return v

    @field_validator("gateway")
    @classmethod
    def _gateway(cls, v):
        if v is True:
            raise ValueError("The `gateway` property must be a string or boolean `false`, not boolean `true`")
        return v

    @model_validator(mode="after")
    def _scaling(self):
        if self.replicas.min != self.replicas.max and not self.scaling:
            raise ValueError("When you set `replicas` to a range, ensure to specify `scaling`.")
        if self.replicas.min == self.replicas.max and self.scaling:
            raise ValueError("To use `scaling`, `replicas` must be set to a range.")
        if not self.commands and not self.image:
            raise ValueError("Either `commands` or `image` must be set")
        return self


AnyRunConfiguration = Annotated[
    Union[DevEnvironmentConfiguration, TaskConfiguration, ServiceConfiguration], Field(discriminator="type")
]
AnyApplyConfiguration = Annotated[
    Union[
        DevEnvironmentConfiguration, TaskConfiguration, ServiceConfiguration, FleetConfiguration,
        GatewayConfiguration, VolumeConfiguration,
    ],
    Field(discriminator="type"),
]

_RUN_ADAPTER = TypeAdapter(AnyRunConfiguration)
_APPLY_ADAPTER = TypeAdapter(AnyApplyConfiguration)


def parse_run_configuration(data: dict):
    try:
        return _RUN_ADAPTER.validate_python(data)
    except ValidationError as e:
        raise ConfigurationError(str(e))


def parse_apply_configuration(data: dict):
    if not isinstance(data, dict) or "type" not in data:
        raise ConfigurationError("configuration must be a mapping with a `type` field")
    try:
        return _APPLY_ADAPTER.validate_python(data)
    except ValidationError as e:
        raise ConfigurationError(str(e))


def is_run_configuration(conf) -> bool:
    return isinstance(conf, (DevEnvironmentConfiguration, TaskConfiguration, ServiceConfiguration))


def apply_configuration_json_schema() -> dict:
    return _APPLY_ADAPTER.json_schema()
