"""Gateways (reference: ``C/models/gateways.py:46-110``)."""

from __future__ import annotations

import datetime
from enum import Enum
from typing import Literal, Optional, Union

from pydantic import Field
from typing_extensions import Annotated

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import CoreModel


class GatewayStatus(str, Enum):
    SUBMITTED = "submitted"
    PROVISIONING = "provisioning"
    RUNNING = "running"
    FAILED = "failed"


class LetsEncryptGatewayCertificate(CoreModel):
    type: Literal["lets-encrypt"] = "lets-encrypt"


class ACMGatewayCertificate(CoreModel):
    type: Literal["acm"] = "acm"
    arn: str


AnyGatewayCertificate = Annotated[
    Union[LetsEncryptGatewayCertificate, ACMGatewayCertificate], Field(discriminator="type")
]


class GatewayConfiguration(CoreModel):
    type: Literal["gateway"] = "gateway"
    name: Optional[str] = None
    default: bool = False
    backend: BackendType
    region: str
    domain: Optional[str] = None
    public_ip: bool = True
    certificate: Optional[AnyGatewayCertificate] = Field(default_factory=LetsEncryptGatewayCertificate)


class GatewaySpec(CoreModel):
    configuration: GatewayConfiguration
    configuration_path: Optional[str] = None


class Gateway(CoreModel):
    name: str
    configuration: GatewayConfiguration
    created_at: datetime.datetime
    status: GatewayStatus
    status_message: Optional[str] = None
    hostname: Optional[str] = None
    ip_address: Optional[str] = None
    instance_id: Optional[str] = None
    backend: BackendType
    region: str
    default: bool = False
    wildcard_domain: Optional[str] = None


class GatewayPlan(CoreModel):
    project_name: str
    user: str
    spec: GatewaySpec
    current_resource: Optional[Gateway] = None


class GatewayComputeConfiguration(CoreModel):
    project_name: str
    instance_name: str
    backend: BackendType
    region: str
    public_ip: bool
    ssh_key_pub: str
    certificate: Optional[AnyGatewayCertificate] = None


class GatewayProvisioningData(CoreModel):
    instance_id: str
    ip_address: str
    region: str
    availability_zone: Optional[str] = None
    hostname: Optional[str] = None
    backend_data: Optional[str] = None
