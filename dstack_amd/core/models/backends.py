"""Backend types and capability sets (reference: ``C/models/backends/base.py:7-41``,
``C/backends/__init__.py:1-37``)."""

from __future__ import annotations

from enum import Enum
from typing import List, Optional

from dstack_amd.core.models.common import CoreModel


class BackendType(str, Enum):
    AWS = "aws"
    AZURE = "azure"
    CUDO = "cudo"
    DATACRUNCH = "datacrunch"
    DSTACK = "dstack"
    GCP = "gcp"
    KUBERNETES = "kubernetes"
    LAMBDA = "lambda"
    LOCAL = "local"
    REMOTE = "remote"  # SSH fleets (on-prem MI355X nodes)
    NEBIUS = "nebius"
    OCI = "oci"
    RUNPOD = "runpod"
    TENSORDOCK = "tensordock"
    VASTAI = "vastai"
    VULTR = "vultr"


BACKENDS_WITH_MULTINODE_SUPPORT = [
    BackendType.AWS, BackendType.AZURE, BackendType.GCP, BackendType.REMOTE, BackendType.OCI,
    BackendType.VULTR, BackendType.LOCAL,
]
BACKENDS_WITH_CREATE_INSTANCE_SUPPORT = [
    BackendType.AWS, BackendType.DSTACK, BackendType.AZURE, BackendType.CUDO, BackendType.DATACRUNCH,
    BackendType.GCP, BackendType.LAMBDA, BackendType.OCI, BackendType.TENSORDOCK, BackendType.VULTR,
    BackendType.LOCAL,
]
BACKENDS_WITH_PLACEMENT_GROUPS_SUPPORT = [BackendType.AWS]
BACKENDS_WITH_RESERVATION_SUPPORT = [BackendType.AWS]
BACKENDS_WITH_GATEWAY_SUPPORT = [BackendType.AWS, BackendType.AZURE, BackendType.GCP, BackendType.KUBERNETES,
                                 BackendType.LOCAL]
# gateways without a public IP (reached from inside the VPC), reference: AWS only
BACKENDS_WITH_PRIVATE_GATEWAY_SUPPORT = [BackendType.AWS, BackendType.LOCAL]
# SSH fleets (remote) have no network-volume API: they use instance mounts (``/host/path:/path``)
BACKENDS_WITH_VOLUMES_SUPPORT = [BackendType.AWS, BackendType.GCP, BackendType.LOCAL, BackendType.RUNPOD]
BACKENDS_WITH_PRIVILEGED_SUPPORT = [b for b in BackendType if b not in (BackendType.RUNPOD, BackendType.VASTAI)]
BACKENDS_WITH_INSTANCE_VOLUMES_SUPPORT = [b for b in BackendType if b not in (BackendType.RUNPOD, BackendType.VASTAI,
                                                                              BackendType.KUBERNETES)]


class ConfigElementValue(CoreModel):
    value: str
    label: str


class ConfigElement(CoreModel):
    selected: Optional[str] = None
    values: List[ConfigElementValue] = []


class ConfigMultiElement(CoreModel):
    selected: List[str] = []
    values: List[ConfigElementValue] = []


class BackendInfo(CoreModel):
    name: BackendType
    config: dict = {}
