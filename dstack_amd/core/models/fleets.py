"""Fleets: cloud instance groups and on-prem SSH fleets (reference: ``C/models/fleets.py:42-291``).

An SSH fleet of 8×MI355X nodes is the primary on-prem target: ``blocks: auto`` splits each node
into GPU blocks aligned to its xGMI topology (see ``server/services/offers.py``).
"""

from __future__ import annotations

import ipaddress
import uuid
from datetime import datetime
from enum import Enum
from typing import List, Literal, Optional, Union

from pydantic import Field, field_validator, model_validator

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import CoreModel
from dstack_amd.core.models.envs import Env
from dstack_amd.core.models.instances import (
    InstanceOfferWithAvailability,
    InstanceStatus,
    InstanceType,
    SSHKey,
)
from dstack_amd.core.models.profiles import (
    PROFILE_PARAM_NAMES,
    Profile,
    ProfileRetry,
    SpotPolicy,
    TerminationPolicy,
    parse_duration,
    parse_idle_duration,
)
from dstack_amd.core.models.resources import IntRange, ResourcesSpec


class FleetStatus(str, Enum):
    SUBMITTED = "submitted"
    ACTIVE = "active"
    TERMINATING = "terminating"
    TERMINATED = "terminated"
    FAILED = "failed"


class InstanceGroupPlacement(str, Enum):
    ANY = "any"
    CLUSTER = "cluster"


def _private_ip(v: Optional[str]) -> Optional[str]:
    if v is None:
        return v
    try:
        ip = ipaddress.ip_address(v)
    except ValueError as e:
        raise ValueError("Invalid IP address") from e
    if not ip.is_private:
        raise ValueError("IP address is not private")
    return v


class SSHHostParams(CoreModel):
    hostname: str
    port: Optional[int] = None
    user: Optional[str] = None
    identity_file: Optional[str] = None
    ssh_key: Optional[SSHKey] = None
    internal_ip: Optional[str] = None
    blocks: Union[Literal["auto"], int] = 1

    _ip = field_validator("internal_ip")(classmethod(lambda cls, v: _private_ip(v)))

    @field_validator("blocks")
    @classmethod
    def _blocks(cls, v):
        if isinstance(v, int) and v < 1:
            raise ValueError("blocks must be >= 1")
        return v


class SSHParams(CoreModel):
    user: Optional[str] = None
    port: Optional[int] = None
    identity_file: Optional[str] = None
    ssh_key: Optional[SSHKey] = None
    hosts: List[Union[SSHHostParams, str]]
    network: Optional[str] = None

    @field_validator("network")
    @classmethod
    def _network(cls, v):
        if v is None:
            return v
        try:
            net = ipaddress.ip_network(v, strict=False)
        except ValueError as e:
            raise ValueError(f"Failed to parse network: {v}") from e
        if not net.is_private:
            raise ValueError("Public network is specified when private network is required")
        return v


class InstanceGroupParams(CoreModel):
    env: Env = Field(default_factory=Env)
    ssh_config: Optional[SSHParams] = None
    nodes: Optional[IntRange] = None
    placement: Optional[InstanceGroupPlacement] = None
    reservation: Optional[str] = None
    resources: Optional[ResourcesSpec] = Field(default_factory=ResourcesSpec)
    blocks: Union[Literal["auto"], int] = 1
    backends: Optional[List[BackendType]] = None
    regions: Optional[List[str]] = None
    instance_types: Optional[List[str]] = None
    spot_policy: Optional[SpotPolicy] = None
    retry: Optional[Union[ProfileRetry, bool]] = None
    max_price: Optional[float] = None
    idle_duration: Optional[Union[Literal["off"], str, int]] = None
    termination_policy: Optional[TerminationPolicy] = None
    termination_idle_time: Optional[Union[str, int]] = None

    @field_validator("nodes", mode="before")
    @classmethod
    def _nodes(cls, v):
        if isinstance(v, int) and not isinstance(v, bool):
            return IntRange(min=v, max=v)
        return v

    @field_validator("idle_duration", mode="before")
    @classmethod
    def _idle(cls, v):
        return parse_idle_duration(v)

    @field_validator("termination_idle_time", mode="before")
    @classmethod
    def _tit(cls, v):
        return parse_duration(v)

    @model_validator(mode="after")
    def _check(self):
        if self.ssh_config is None and self.nodes is None:
            raise ValueError("Either `nodes` or `ssh_config` must be set")
        if self.ssh_config is not None and self.nodes is not None:
            raise ValueError("`nodes` and `ssh_config` are mutually exclusive")
        return self


class FleetConfiguration(InstanceGroupParams):
    type: Literal["fleet"] = "fleet"
    name: Optional[str] = None


class FleetSpec(CoreModel):
    configuration: FleetConfiguration
    configuration_path: Optional[str] = None
    profile: Profile = Field(default_factory=lambda: Profile(name="default"))
    autocreated: bool = False

    @property
    def merged_profile(self) -> Profile:
        merged = self.profile.model_copy(deep=True)
        for key in PROFILE_PARAM_NAMES:
            val = getattr(self.configuration, key, None)
            if val is not None:
                setattr(merged, key, val)
        if merged.spot_policy is None:
            merged.spot_policy = SpotPolicy.ONDEMAND
        if merged.retry is None:
            merged.retry = False
        return merged


class Instance(CoreModel):
    id: uuid.UUID
    project_name: str
    backend: Optional[BackendType] = None
    instance_type: Optional[InstanceType] = None
    name: str
    fleet_id: Optional[uuid.UUID] = None
    fleet_name: Optional[str] = None
    instance_num: int = 0
    pool_name: Optional[str] = None
    job_name: Optional[str] = None
    hostname: Optional[str] = None
    status: InstanceStatus
    unreachable: bool = False
    termination_reason: Optional[str] = None
    created: datetime
    region: Optional[str] = None
    price: Optional[float] = None
    total_blocks: Optional[int] = None
    busy_blocks: int = 0
    health: Optional[dict] = None


class Fleet(CoreModel):
    id: Optional[uuid.UUID] = None
    name: str
    project_name: str
    spec: FleetSpec
    created_at: datetime
    status: FleetStatus
    status_message: Optional[str] = None
    instances: List[Instance] = []


class FleetPlan(CoreModel):
    project_name: str
    user: str
    spec: FleetSpec
    current_resource: Optional[Fleet] = None
    offers: List[InstanceOfferWithAvailability] = []
    total_offers: int = 0
    max_offer_price: Optional[float] = None


class Pool(CoreModel):
    name: str
    default: bool
    created_at: datetime
    total_instances: int
    available_instances: int


class PoolInstances(CoreModel):
    name: str
    instances: List[Instance]
