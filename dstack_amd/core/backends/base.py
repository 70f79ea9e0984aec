"""Backend Compute interface and shared bootstrap helpers (reference:
``C/backends/base/compute.py:45-451``, ``C/backends/base/offers.py:18-175``)."""

from __future__ import annotations

import threading
import time
from abc import ABC, abstractmethod
from typing import Dict, List, Optional, Tuple

from dstack_amd.core.errors import BackendError, ComputeError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.gateways import GatewayComputeConfiguration, GatewayProvisioningData
from dstack_amd.core.models.instances import (
    InstanceAvailability,
    InstanceConfiguration,
    InstanceOffer,
    InstanceOfferWithAvailability,
)
from dstack_amd.core.models.placement import PlacementGroup, PlacementGroupProvisioningData
from dstack_amd.core.models.resources import ResourcesSpec
from dstack_amd.core.models.runs import Job, JobProvisioningData, Requirements, Run
from dstack_amd.core.models.volumes import Volume, VolumeAttachmentData, VolumeProvisioningData

DSTACK_SHIM_HTTP_PORT = 10998
DSTACK_RUNNER_HTTP_PORT = 10999
DSTACK_RUNNER_SSH_PORT = 10022
OFFERS_CACHE_TTL = 30.0


class Compute(ABC):
    TYPE: BackendType

    def __init__(self):
        self._offers_cache: Dict[str, Tuple[float, List[InstanceOfferWithAvailability]]] = {}
        self._offers_lock = threading.Lock()

    # ---- offers ----------------------------------------------------------------------------
    @abstractmethod
    def get_offers(self, requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
        ...

    def get_offers_cached(self, requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
        key = requirements.model_dump_json() if requirements else ""
        with self._offers_lock:
            hit = self._offers_cache.get(key)
            if hit and time.monotonic() - hit[0] < OFFERS_CACHE_TTL:
                return hit[1]
        offers = self.get_offers(requirements)
        with self._offers_lock:
            self._offers_cache[key] = (time.monotonic(), offers)
        return offers

    # ---- instances ---------------------------------------------------------------------------
    def run_job(self, run: Run, job: Job, instance_offer: InstanceOfferWithAvailability,
                project_ssh_public_key: str, project_ssh_private_key: str,
                volumes: List[Volume]) -> JobProvisioningData:
        """Provision an instance for one job (default: create_instance with a job-derived config)."""
        from dstack_amd.core.models.instances import SSHKey

        cfg = InstanceConfiguration(
            project_name=run.project_name, instance_name=f"{run.run_spec.run_name}-{job.job_spec.job_num}",
            user=run.user, ssh_keys=[SSHKey(public=project_ssh_public_key.strip())], volumes=volumes,
        )
        return self.create_instance(instance_offer, cfg)

    def create_instance(self, instance_offer: InstanceOfferWithAvailability,
                        instance_config: InstanceConfiguration) -> JobProvisioningData:
        raise NotImplementedError(f"{self.TYPE.value} cannot create instances")

    @abstractmethod
    def terminate_instance(self, instance_id: str, region: str, backend_data: Optional[str] = None) -> None:
        ...

    def update_provisioning_data(self, provisioning_data: JobProvisioningData, project_ssh_public_key: str,
                                 project_ssh_private_key: str) -> None:
        """Fill hostname/internal_ip once the cloud reports them (no-op when already set)."""

    # ---- placement groups --------------------------------------------------------------------
    def create_placement_group(self, placement_group: PlacementGroup) -> PlacementGroupProvisioningData:
        raise NotImplementedError()

    def delete_placement_group(self, placement_group: PlacementGroup) -> None:
        raise NotImplementedError()

    # ---- gateways ----------------------------------------------------------------------------
    def create_gateway(self, configuration: GatewayComputeConfiguration) -> GatewayProvisioningData:
        raise NotImplementedError()

    def terminate_gateway(self, instance_id: str, configuration: GatewayComputeConfiguration,
                          backend_data: Optional[str] = None) -> None:
        raise NotImplementedError()

    # ---- volumes -----------------------------------------------------------------------------
    def register_volume(self, volume: Volume) -> VolumeProvisioningData:
        raise NotImplementedError()

    def create_volume(self, volume: Volume) -> VolumeProvisioningData:
        raise NotImplementedError()

    def delete_volume(self, volume: Volume) -> None:
        raise NotImplementedError()

    def attach_volume(self, volume: Volume, instance_id: str) -> VolumeAttachmentData:
        raise NotImplementedError()

    def detach_volume(self, volume: Volume, instance_id: str, force: bool = False) -> None:
        raise NotImplementedError()

    def is_volume_detached(self, volume: Volume, instance_id: str) -> bool:
        return True


def offer_matches(offer: InstanceOffer, req: Optional[Requirements]) -> bool:
    """Catalog matching (reference ``match_requirements``)."""
    if req is None:
        return True
    r: ResourcesSpec = req.resources
    res = offer.instance.resources
    if not r.cpu.contains(res.cpus):
        return False
    if not r.memory.contains(res.memory_mib / 1024):
        return False
    if r.disk and r.disk.size.max is not None and res.disk.size_mib / 1024 < r.disk.size.min:
        return False
    if req.spot is not None and res.spot != req.spot:
        return False
    if req.max_price is not None and offer.price > req.max_price:
        return False
    g = r.gpu
    if g is None or (g.count.max == 0):
        return not res.gpus if (g is not None and g.count.max == 0) else True
    if not g.count.contains(len(res.gpus)):
        return False
    if not res.gpus:
        return g.count.min == 0
    gpu = res.gpus[0]
    if g.vendor is not None and gpu.vendor is not None and gpu.vendor != g.vendor:
        return False
    if g.name and gpu.name.lower() not in {n.lower() for n in g.name}:
        return False
    if g.memory is not None and not g.memory.contains(gpu.memory_mib / 1024):
        return False
    if g.total_memory is not None and not g.total_memory.contains(gpu.memory_mib / 1024 * len(res.gpus)):
        return False
    return True


def choose_disk_size_mib(req: Optional[Requirements], default_gb: int = 100) -> int:
    if req is None or req.resources.disk is None:
        return default_gb * 1024
    size = req.resources.disk.size
    gb = size.min if size.min is not None else default_gb
    return int(gb * 1024)


def with_availability(offers: List[InstanceOffer], availability=InstanceAvailability.AVAILABLE):
    return [InstanceOfferWithAvailability(**o.model_dump(), availability=availability) for o in offers]


# ---------------------------------------------------------------------------------------------
# bootstrap scripts (cloud-init / SSH deploy)
# ---------------------------------------------------------------------------------------------
def get_shim_env(authorized_keys: List[str], runner_url: str = "", shim_http_port: int = DSTACK_SHIM_HTTP_PORT,
                 driver: str = "auto") -> Dict[str, str]:
    return {
        "DSTACK_SHIM_HTTP_PORT": str(shim_http_port),
        "DSTACK_RUNNER_HTTP_PORT": str(DSTACK_RUNNER_HTTP_PORT),
        "DSTACK_RUNNER_SSH_PORT": str(DSTACK_RUNNER_SSH_PORT),
        "DSTACK_RUNNER_DOWNLOAD_URL": runner_url,
        "DSTACK_SHIM_DRIVER": driver,
        "DSTACK_PUBLIC_SSH_KEY": "\n".join(authorized_keys),
    }


def get_shim_commands(authorized_keys: List[str], shim_url: str, runner_url: str, is_privileged: bool = False,
                      driver: str = "auto") -> List[str]:
    """Commands a fresh VM runs (cloud-init) to fetch and start the shim (compute.py:216-309)."""
    env = get_shim_env(authorized_keys, runner_url, driver=driver)
    exports = " ".join(f"{k}='{v}'" for k, v in env.items() if k != "DSTACK_PUBLIC_SSH_KEY")
    return [
        "mkdir -p /root/.dstack-shim",
        f"curl -fsSL -o /usr/local/bin/dstack-shim '{shim_url}' && chmod +x /usr/local/bin/dstack-shim",
        f"curl -fsSL -o /root/.dstack-shim/dstack-runner '{runner_url}' && chmod +x /root/.dstack-shim/dstack-runner",
        f"{exports} nohup /usr/local/bin/dstack-shim --service --driver {driver}"
        + (" --privileged" if is_privileged else "")
        + " > /root/.dstack-shim/shim.log 2>&1 &",
    ]


# amdgpu-install releases used when a GPU host boots without the kernel driver (the ROCm user space
# ships in the job's container image; the host only needs amdgpu + /dev/kfd).  MI350X/MI355X
# (gfx950) need the ROCm 7.x driver; the earlier Instinct parts are served by 6.4.
AMDGPU_INSTALL_RELEASES = {
    "gfx950": ("7.0", "amdgpu-install_7.0.70000-1_all.deb"),
    "default": ("6.4", "amdgpu-install_6.4.60400-1_all.deb"),
}
AMDGPU_INSTALL_RELEASE, AMDGPU_INSTALL_DEB = AMDGPU_INSTALL_RELEASES["default"]
# PCI device ids of the Instinct GPUs this build schedules (MI100 .. MI355X), vendor 1002
AMD_INSTINCT_PCI = "738c|740c|740f|74a0|74a1|74a5|74b5|75a0|75a3"
AMD_GFX950_PCI = "75a0|75a3"  # MI350X, MI355X
# written when the bootstrap could not bring up /dev/kfd; the shim reports its text in host_info
# ("gpu_driver_error") and the server fails the instance's provisioning with it
AMDGPU_FAILED_MARKER = "/var/lib/dstack/amdgpu-install.failed"


def get_amd_driver_commands(releases: Optional[Dict[str, tuple]] = None, marker: str = AMDGPU_FAILED_MARKER,
                            log: str = "/var/log/dstack-amdgpu.log", os_release: str = "/etc/os-release") -> List[str]:
    """Host setup for clouds whose default image has no AMD GPU driver (plain Ubuntu on AWS, GCP,
    Azure, OCI...): when the host has an Instinct GPU but no ``/dev/kfd``, install the amdgpu DKMS
    driver with amdgpu-install and load it, before the shim starts (it discovers GPUs through KFD).

    * the release follows the detected part (``AMDGPU_INSTALL_RELEASES``: 7.x for gfx950);
    * the Ubuntu codename comes from ``/etc/os-release`` (jammy, noble, ...), not a fixed one;
    * the running kernel's headers are installed first (DKMS builds against them);
    * when ``/dev/kfd`` is still missing afterwards, ``marker`` gets the reason and the log tail,
      so the host fails provisioning with it instead of registering with zero GPUs.

    A no-op on hosts that already have the driver (vendor GPU images, the packer image in
    ``scripts/packer``) and on CPU hosts.  The reference ships its own VM images instead."""
    rel = dict(AMDGPU_INSTALL_RELEASES, **(releases or {}))
    new_rel, new_deb = rel["gfx950"]
    old_rel, old_deb = rel["default"]
    script = (
        f"if lspci -nn 2>/dev/null | grep -qiE '1002:({AMD_INSTINCT_PCI})' && [ ! -e /dev/kfd ]; then "
        f"export DEBIAN_FRONTEND=noninteractive; rm -f {marker}; "
        f"CODENAME=$(. {os_release} 2>/dev/null; echo ${{VERSION_CODENAME:-${{UBUNTU_CODENAME:-jammy}}}}); "
        f"if lspci -nn | grep -qiE '1002:({AMD_GFX950_PCI})'; then REL={new_rel}; DEB={new_deb}; "
        f"else REL={old_rel}; DEB={old_deb}; fi; "
        f"echo \"amdgpu-install $REL for ubuntu/$CODENAME on kernel $(uname -r)\"; "
        f"apt-get update -qq; apt-get install -yqq \"linux-headers-$(uname -r)\"; "
        f"curl -fsSL -o /tmp/amdgpu-install.deb \"https://repo.radeon.com/amdgpu-install/$REL/ubuntu/$CODENAME/$DEB\" "
        f"&& apt-get install -yqq /tmp/amdgpu-install.deb && amdgpu-install -y --usecase=dkms --no-32 "
        f"&& modprobe amdgpu; "
        f"if [ ! -e /dev/kfd ]; then mkdir -p $(dirname {marker}); "
        f"{{ echo \"amdgpu $REL driver install failed on ubuntu/$CODENAME kernel $(uname -r): /dev/kfd missing\"; "
        f"tail -n 5 {log}; }} > {marker} 2>/dev/null; fi; "
        f"fi >> {log} 2>&1"
    )
    return [script]


def get_user_data(authorized_keys: List[str], shim_url: str, runner_url: str,
                  backend_commands: Optional[List[str]] = None) -> str:
    """cloud-config: authorized keys, then the cloud's own host setup (``backend_commands``, e.g.
    opening the VPC subnet in the host firewall), the AMD driver when the image lacks it, then the
    shim bootstrap."""
    cmds = (list(backend_commands or []) + get_amd_driver_commands()
            + get_shim_commands(authorized_keys, shim_url, runner_url))
    keys = "\n".join(f"  - {json_quote(k)}" for k in authorized_keys)  # a YAML-safe scalar whatever the comment
    runcmd = "\n".join(f"  - {json_quote(c)}" for c in cmds)
    return f"#cloud-config\nssh_authorized_keys:\n{keys}\nruncmd:\n{runcmd}\n"


def json_quote(s: str) -> str:
    import json

    return json.dumps(s)


def get_docker_commands(authorized_keys: List[str], runner_url: str) -> List[str]:
    """Container-only backends (runpod/vastai/k8s): install sshd and start the runner directly
    (compute.py:334-387)."""
    import shlex

    keys = shlex.quote("".join(k + "\n" for k in authorized_keys))  # comments may hold quotes
    return [
        "export DEBIAN_FRONTEND=noninteractive",
        "(command -v sshd || (apt-get update -qq && apt-get install -yqq openssh-server)) >/dev/null 2>&1",
        "mkdir -p ~/.ssh /run/sshd && chmod 700 ~/.ssh",
        f"printf '%s' {keys} >> ~/.ssh/authorized_keys && chmod 600 ~/.ssh/authorized_keys",
        f"$(command -v sshd) -p {DSTACK_RUNNER_SSH_PORT} -o PermitUserEnvironment=yes",
        f"curl -fsSL -o /usr/local/bin/dstack-runner '{runner_url}' && chmod +x /usr/local/bin/dstack-runner",
        f"/usr/local/bin/dstack-runner start --http-port {DSTACK_RUNNER_HTTP_PORT} --temp-dir /tmp/runner "
        "--home-dir /root --working-dir /workflow --ssh-env",
    ]


def raise_compute_error(msg: str):
    raise ComputeError(msg)


class BackendUnavailable(BackendError):
    pass
