"""Volumes: network volumes and instance (host path) mounts (reference: ``C/models/volumes.py``).

MI355X sizing note: a Llama-3-70B bf16 checkpoint (~140 GB) plus optimizer shards for 8 GPUs fit a
single 2 TB volume; ``recommended_volume_size_gb`` sizes per-replica volumes from the 288 GB/GPU
HBM so that a full device-memory dump (checkpoint/resume) always fits.
"""

from __future__ import annotations

import uuid
from datetime import datetime
from enum import Enum
from pathlib import PurePosixPath
from typing import List, Literal, Optional, Tuple, Union

from pydantic import Field, field_validator

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import CoreModel
from dstack_amd.core.models.resources import Memory


class VolumeStatus(str, Enum):
    SUBMITTED = "submitted"
    PROVISIONING = "provisioning"
    ACTIVE = "active"
    FAILED = "failed"

    def is_active(self) -> bool:
        return self not in self.finished_statuses()

    @classmethod
    def finished_statuses(cls) -> List["VolumeStatus"]:
        return [cls.FAILED]


class VolumeConfiguration(CoreModel):
    type: Literal["volume"] = "volume"
    name: Optional[str] = None
    backend: BackendType
    region: str
    size: Optional[Memory] = Field(None, description="Required when creating a new volume")
    volume_id: Optional[str] = Field(None, description="Required when registering an external volume")

    @property
    def size_gb(self) -> int:
        if self.size is None:
            raise ValueError("volume size is not set")
        return int(self.size)


class VolumeSpec(CoreModel):
    configuration: VolumeConfiguration
    configuration_path: Optional[str] = None


class VolumeProvisioningData(CoreModel):
    backend: Optional[BackendType] = None
    volume_id: str
    size_gb: int
    availability_zone: Optional[str] = None
    price: Optional[float] = None
    attachable: bool = True
    detachable: bool = True
    backend_data: Optional[str] = None


class VolumeAttachmentData(CoreModel):
    device_name: Optional[str] = None


class Volume(CoreModel):
    id: uuid.UUID
    name: str
    user: str = ""
    project_name: str
    configuration: VolumeConfiguration
    external: bool
    created_at: datetime
    status: VolumeStatus
    status_message: Optional[str] = None
    deleted: bool = False
    volume_id: Optional[str] = None
    provisioning_data: Optional[VolumeProvisioningData] = None
    attachment_data: Optional[VolumeAttachmentData] = None


class VolumePlan(CoreModel):
    project_name: str
    user: str
    spec: VolumeSpec
    current_resource: Optional[Volume] = None


def _validate_path(path: str) -> str:
    if not path:
        raise ValueError("empty path")
    p = PurePosixPath(path)
    if not p.is_absolute():
        raise ValueError(f"path must be absolute: {path}")
    if ".." in p.parts:
        raise ValueError(f".. are not allowed: {path}")
    return str(p)


def _split(mount_point: str) -> Tuple[str, str]:
    parts = mount_point.split(":")
    if len(parts) != 2:
        raise ValueError(f"invalid mount point format: {mount_point}")
    return parts[0], parts[1]


class VolumeMountPoint(CoreModel):
    name: Union[str, List[str]] = Field(..., description="Network volume name (or alternatives)")
    path: str

    _vp = field_validator("path")(classmethod(lambda cls, v: _validate_path(v)))

    @classmethod
    def parse(cls, v: str) -> "VolumeMountPoint":
        name, path = _split(v)
        return cls(name=name, path=path)


class InstanceMountPoint(CoreModel):
    instance_path: str
    path: str
    optional: bool = False

    _vip = field_validator("instance_path", "path")(classmethod(lambda cls, v: _validate_path(v)))

    @classmethod
    def parse(cls, v: str) -> "InstanceMountPoint":
        ip, path = _split(v)
        return cls(instance_path=ip, path=path)


MountPoint = Union[VolumeMountPoint, InstanceMountPoint]


def parse_mount_point(v: Union[str, dict, VolumeMountPoint, InstanceMountPoint]) -> MountPoint:
    if isinstance(v, (VolumeMountPoint, InstanceMountPoint)):
        return v
    if isinstance(v, dict):
        if "instance_path" in v:
            return InstanceMountPoint.model_validate(v)
        return VolumeMountPoint.model_validate(v)
    src, dest = _split(v)
    if "/" in src:
        return InstanceMountPoint(instance_path=src, path=dest)
    return VolumeMountPoint(name=src, path=dest)


def recommended_volume_size_gb(gpus_per_replica: int, hbm_gb_per_gpu: float = 288.0, headroom: float = 1.5) -> int:
    """Volume size that holds a full-HBM checkpoint of every GPU of a replica, with headroom."""
    return int(max(100, gpus_per_replica * hbm_gb_per_gpu * headroom))
