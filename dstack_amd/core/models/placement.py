"""Placement groups (reference: ``C/models/placement.py``)."""

from __future__ import annotations

from enum import Enum
from typing import Optional

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import CoreModel


class PlacementStrategy(str, Enum):
    CLUSTER = "cluster"


class PlacementGroupConfiguration(CoreModel):
    backend: BackendType
    region: str
    placement_strategy: PlacementStrategy = PlacementStrategy.CLUSTER


class PlacementGroupProvisioningData(CoreModel):
    backend: BackendType
    backend_data: Optional[str] = None


class PlacementGroup(CoreModel):
    name: str
    project_name: str
    configuration: PlacementGroupConfiguration
    provisioning_data: Optional[PlacementGroupProvisioningData] = None
