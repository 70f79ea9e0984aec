"""Instances, offers and host topology (reference: ``C/models/instances.py:14-167``).

MI355X addition: ``HostTopology`` carries the amdsmi view of a node — per-GPU BDF, render node,
HBM size and the xGMI link matrix — so the scheduler can hand out fully-connected GPU sets and
align ``blocks`` to xGMI sub-meshes.
"""

from __future__ import annotations

from enum import Enum
from typing import Dict, List, Optional

from pydantic import Field, model_validator

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import CoreModel
from dstack_amd.core.models.envs import Env
from dstack_amd.core.models.resources import AcceleratorVendor


class Gpu(CoreModel):
    name: str
    memory_mib: int
    vendor: Optional[AcceleratorVendor] = None

    @model_validator(mode="before")
    @classmethod
    def _vendor(cls, values):
        if isinstance(values, dict):
            values = dict(values)
            name = values.get("name") or ""
            if name.startswith("tpu-"):
                values["name"] = name[4:]
                values.setdefault("vendor", AcceleratorVendor.GOOGLE)
            if values.get("vendor") is None:
                from dstack_amd.core.models.gpus import vendor_of

                values["vendor"] = vendor_of(values.get("name", "")) or AcceleratorVendor.NVIDIA
            elif isinstance(values["vendor"], str):
                values["vendor"] = AcceleratorVendor.cast(values["vendor"])
        return values


class Disk(CoreModel):
    size_mib: int


class Resources(CoreModel):
    cpus: int
    memory_mib: int
    gpus: List[Gpu] = []
    spot: bool = False
    disk: Disk = Field(default_factory=lambda: Disk(size_mib=102400))
    description: str = ""

    def pretty_format(self, include_spot: bool = False) -> str:
        parts = []
        if self.cpus > 0:
            parts.append(f"{self.cpus}xCPU")
        if self.memory_mib > 0:
            parts.append(f"{self.memory_mib / 1024:.0f}GB")
        if self.gpus:
            g = self.gpus[0]
            s = f"{len(self.gpus)}x{g.name}"
            if g.memory_mib > 0:
                s += f" ({g.memory_mib / 1024:.0f}GB)"
            parts.append(s)
        if self.disk.size_mib > 0:
            parts.append(f"{self.disk.size_mib / 1024:.1f}GB (disk)")
        out = ", ".join(parts)
        if include_spot and self.spot:
            out += ", SPOT"
        return out


class InstanceType(CoreModel):
    name: str
    resources: Resources


class GpuDevice(CoreModel):
    """One accelerator as discovered on a host by the shim (amdsmi)."""

    index: int
    name: str
    vendor: AcceleratorVendor = AcceleratorVendor.AMD
    memory_mib: int = 0
    bdf: Optional[str] = None
    render_node: Optional[str] = None  # /dev/dri/renderD<N> (the AMD lock/resource id)
    arch: Optional[str] = None  # gfx950
    serial: Optional[str] = None


class HostTopology(CoreModel):
    gpus: List[GpuDevice] = []
    # xgmi[i][j] = number of direct xGMI links between GPU i and j (0 = routed / PCIe)
    xgmi: List[List[int]] = []
    numa: Dict[int, int] = {}  # gpu index -> NUMA node
    nics: List[str] = []  # RDMA-capable NICs (RoCE/IB) for inter-node RCCL

    def fully_connected(self, subset: List[int]) -> bool:
        if not self.xgmi:
            return False
        return all(self.xgmi[a][b] > 0 for a in subset for b in subset if a != b)


class SSHConnectionParams(CoreModel):
    hostname: str
    username: str
    port: int

    model_config = {**CoreModel.model_config, "frozen": True}


class SSHKey(CoreModel):
    public: str
    private: Optional[str] = None


class RemoteConnectionInfo(CoreModel):
    host: str
    port: int
    ssh_user: str
    ssh_keys: List[SSHKey]
    env: Env = Field(default_factory=Env)


class InstanceConfiguration(CoreModel):
    project_name: str
    instance_name: str
    user: str
    ssh_keys: List[SSHKey]
    instance_id: Optional[str] = None
    availability_zone: Optional[str] = None
    placement_group_name: Optional[str] = None
    reservation: Optional[str] = None
    volumes: Optional[list] = None

    def get_public_keys(self) -> List[str]:
        return [k.public.strip() for k in self.ssh_keys]


class InstanceRuntime(str, Enum):
    SHIM = "shim"
    RUNNER = "runner"


class InstanceAvailability(str, Enum):
    UNKNOWN = "unknown"
    AVAILABLE = "available"
    NOT_AVAILABLE = "not_available"
    NO_QUOTA = "no_quota"
    IDLE = "idle"
    BUSY = "busy"

    def is_available(self) -> bool:
        return self in (InstanceAvailability.UNKNOWN, InstanceAvailability.AVAILABLE, InstanceAvailability.IDLE)


class InstanceOffer(CoreModel):
    backend: BackendType
    instance: InstanceType
    region: str
    price: float


class InstanceOfferWithAvailability(InstanceOffer):
    availability: InstanceAvailability
    instance_runtime: InstanceRuntime = InstanceRuntime.SHIM
    blocks: int = 1
    total_blocks: int = 1


class InstanceStatus(str, Enum):
    PENDING = "pending"
    PROVISIONING = "provisioning"
    IDLE = "idle"
    BUSY = "busy"
    TERMINATING = "terminating"
    TERMINATED = "terminated"

    def is_available(self) -> bool:
        return self in (InstanceStatus.IDLE, InstanceStatus.BUSY)

    def is_active(self) -> bool:
        return self not in self.finished_statuses()

    @classmethod
    def finished_statuses(cls) -> List["InstanceStatus"]:
        return [cls.TERMINATING, cls.TERMINATED]


class InstanceHealth(CoreModel):
    """Result of the HIP health probes run on a host (HBM BW, MFMA TFLOPS, xGMI, RCCL)."""

    healthy: bool = True
    hbm_tb_s: Optional[List[float]] = None
    mfma_bf16_tflops: Optional[List[float]] = None
    mfma_fp8_tflops: Optional[List[float]] = None
    xgmi_gb_s: Optional[List[List[float]]] = None
    rccl_busbw_gb_s: Optional[float] = None
    message: str = ""
    sku: Optional[str] = None  # the part the thresholds are relative to (e.g. MI355X)
    thresholds: Optional[dict] = None  # e.g. {"hbm_tb_s": 4.8, "mfma_bf16_tflops": 1680}
    ran_at: Optional[float] = None  # unix seconds of the probe run
    source: Optional[str] = None  # "shim" (async, off the job path) | "runner" (job pre-flight)
