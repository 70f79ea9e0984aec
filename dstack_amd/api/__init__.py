"""Public Python API (reference: ``src/dstack/api/__init__.py``)."""

from dstack_amd.api._public import (
    Backend,
    BackendCollection,
    Client,
    FleetCollection,
    PoolCollection,
    PoolInstance,
    RepoCollection,
    Run,
    RunCollection,
    VolumeCollection,
)
from dstack_amd.api.server import APIClient
from dstack_amd.core.errors import ClientError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import RegistryAuth
from dstack_amd.core.models.configurations import DevEnvironmentConfiguration as DevEnvironment
from dstack_amd.core.models.configurations import ServiceConfiguration as Service
from dstack_amd.core.models.configurations import TaskConfiguration as Task
from dstack_amd.core.models.repos import LocalRepo, RemoteRepo, VirtualRepo
from dstack_amd.core.models.resources import ComputeCapability, Memory, Range
from dstack_amd.core.models.resources import DiskSpec as Disk
from dstack_amd.core.models.resources import GPUSpec as GPU
from dstack_amd.core.models.resources import ResourcesSpec as Resources
from dstack_amd.core.models.runs import RunStatus
from dstack_amd.core.models.services import OpenAIChatModel, ScalingSpec as Scaling, TGIChatModel
from dstack_amd.core.services.ssh.ports import PortUsedError

__all__ = [
    "APIClient", "Backend", "BackendCollection", "BackendType", "Client", "ClientError", "ComputeCapability", "DevEnvironment", "Disk",
    "FleetCollection", "GPU", "PoolCollection", "PoolInstance", "LocalRepo", "Memory", "OpenAIChatModel", "PortUsedError", "Range", "RegistryAuth",
    "RemoteRepo", "RepoCollection", "Resources", "Run", "RunCollection", "RunStatus", "Scaling", "Service", "Task",
    "TGIChatModel", "VirtualRepo", "VolumeCollection",
]
