"""``local`` backend: runs jobs on the server's own host through a locally started
``dstack-shim`` (process driver), talking to it over loopback HTTP — no SSH (reference:
``C/backends/local/compute.py:21-101``).

Unlike the reference's fake 4 CPU/8 GB offer, the MI355X build offers the host's real resources:
CPU count, memory and the AMD GPUs reported by the shim's amdsmi probe (``dstack-shim --host-info``),
so a local 8×MI355X box can run the headline Llama-3-8B task through ``dstack apply``.
"""

from __future__ import annotations

import json
import os
import subprocess
import threading
import time
from typing import Dict, List, Optional

import httpx

from dstack_amd.core.backends.base import Compute, choose_disk_size_mib, offer_matches
from dstack_amd.core.errors import ComputeError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import (
    Disk,
    Gpu,
    InstanceAvailability,
    InstanceConfiguration,
    InstanceOfferWithAvailability,
    InstanceType,
    Resources,
)
from dstack_amd.core.models.runs import JobProvisioningData, Requirements
from dstack_amd.core.models.volumes import Volume, VolumeProvisioningData
from dstack_amd import native_bin


class LocalShim:
    """The single shim process owned by the server for the local backend -- or, with
    ``DSTACK_LOCAL_SHIM_PER_INSTANCE=1``, one shim per local instance, started by
    ``create_instance`` and stopped by ``terminate_instance`` like a VM's agent, so a fresh
    instance's agent start (``--host-info``, process start, first healthcheck) is in the job's
    cold start (``bench_coldstart.py``).  Per-instance shims do not arbitrate GPUs between each
    other: the mode is for sequential cold-start measurement, the shared shim for everything else."""

    _instance: Optional["LocalShim"] = None
    _lock = threading.Lock()
    _per_instance: Dict[str, "LocalShim"] = {}

    def __init__(self, home: str):
        self.home = home
        self.proc: Optional[subprocess.Popen] = None
        self.port: Optional[int] = None
        self.host_info: dict = {}
        self.timings: Dict[str, float] = {}  # agent start stages (s) of the last start

    @classmethod
    def get(cls) -> "LocalShim":
        with cls._lock:
            if cls._instance is None:
                from dstack_amd.server import settings

                cls._instance = LocalShim(str(settings.SERVER_DIR_PATH / "local-shim"))
            inst = cls._instance
        inst.ensure_started()
        return inst

    def ensure_started(self):
        with self._lock:
            if self.proc is not None and self.proc.poll() is None:
                return
            shim = native_bin.shim_path()
            runner = native_bin.runner_path()
            if not shim or not runner:
                raise ComputeError("native agents are not built (make -C native)")
            os.makedirs(self.home, exist_ok=True)
            t0 = time.perf_counter()
            info = subprocess.run([shim, "--host-info"], capture_output=True, text=True, timeout=60)
            t_info = time.perf_counter()
            try:
                self.host_info = json.loads(info.stdout.strip().splitlines()[-1])
            except (ValueError, IndexError):
                self.host_info = {}
            args = [shim, "--shim-home", self.home, "--shim-http-port", "0", "--host", "127.0.0.1",
                    "--runner-binary-path", runner, "--driver", os.environ.get("DSTACK_LOCAL_SHIM_DRIVER", "process")]
            probe = native_bin.probe_path()
            if probe and os.environ.get("DSTACK_LOCAL_GPU_PROBE") == "1":
                args += ["--probe-binary", probe]
            self.proc = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=open(os.path.join(self.home, "shim.log"), "a"),
                                         text=True, start_new_session=True)
            line = self.proc.stdout.readline()
            if not line.startswith("DSTACK_SHIM_PORT="):
                raise ComputeError(f"local shim failed to start: {line!r}")
            self.port = int(line.strip().split("=", 1)[1])
            t_port = time.perf_counter()
            for _ in range(200):
                try:
                    if httpx.get(f"http://127.0.0.1:{self.port}/api/healthcheck", timeout=1).status_code == 200:
                        break
                except httpx.HTTPError:
                    time.sleep(0.01)
            t_ok = time.perf_counter()
            self.timings = {"host_info_s": round(t_info - t0, 4), "process_start_s": round(t_port - t_info, 4),
                            "first_healthcheck_s": round(t_ok - t_port, 4), "agent_start_s": round(t_ok - t0, 4)}

    def stop(self):
        if self.proc and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()


def host_resources(host_info: dict) -> Resources:
    topo = host_info.get("topology") or {}
    gpus = [
        Gpu(name=g.get("name") or "AMD GPU", memory_mib=int(g.get("memory_mib") or 0), vendor=g.get("vendor") or "amd")
        for g in topo.get("gpus", [])
    ]
    return Resources(
        cpus=int(host_info.get("cpus") or os.cpu_count() or 1),
        memory_mib=int((host_info.get("memory") or 0) / 2**20),
        gpus=gpus,
        spot=False,
        disk=Disk(size_mib=int((host_info.get("disk_size") or 100 * 2**30) / 2**20)),
    )


class LocalCompute(Compute):
    TYPE = BackendType.LOCAL

    def get_offers(self, requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
        shim = LocalShim.get()
        res = host_resources(shim.host_info)
        g = requirements.resources.gpu if requirements is not None else None
        if g is not None and res.gpus and not g.count.contains(len(res.gpus)):
            # the host's shim grants GPU subsets (xGMI-aware lock), so offer as many as the run
            # allows: `gpu: MI355X:1` or two 2-GPU nodes of a multi-node task fit an 8-GPU host
            hi = len(res.gpus) if g.count.max is None else min(len(res.gpus), g.count.max)
            if hi >= max(1, g.count.min or 0):
                res = res.model_copy(update={"gpus": res.gpus[:hi]})
        offer = InstanceOfferWithAvailability(
            backend=BackendType.LOCAL, instance=InstanceType(name="local", resources=res), region="local",
            price=0.0, availability=InstanceAvailability.AVAILABLE,
        )
        if requirements is not None:
            # the local host is one instance: disk/cpu/memory lower bounds are advisory
            req = requirements.model_copy(deep=True)
            req.resources.disk = None
            req.resources.cpu.min = min(req.resources.cpu.min or 0, res.cpus)
            req.resources.memory.min = min(req.resources.memory.min or 0, res.memory_mib / 1024)
            if not offer_matches(offer, req):
                return []
        return [offer]

    def create_instance(self, instance_offer: InstanceOfferWithAvailability,
                        instance_config: InstanceConfiguration) -> JobProvisioningData:
        instance_id = f"local-{instance_config.instance_name}"
        data: dict = {}
        if os.environ.get("DSTACK_LOCAL_SHIM_PER_INSTANCE") == "1":
            from dstack_amd.server import settings

            shim = LocalShim(str(settings.SERVER_DIR_PATH / "local-shims" / instance_config.instance_name))
            shim.ensure_started()  # the agent start of a fresh instance
            LocalShim._per_instance[instance_id] = shim
            data = {"per_instance_shim": True, "agent": shim.timings}
        else:
            shim = LocalShim.get()
        return JobProvisioningData(
            backend=BackendType.LOCAL, instance_type=instance_offer.instance,
            instance_id=instance_id, hostname="127.0.0.1", internal_ip="127.0.0.1",
            region="local", price=0.0, username=os.environ.get("USER", "root"), ssh_port=None, dockerized=True,
            backend_data=json.dumps({"shim_port": shim.port, **data}),
        )

    def terminate_instance(self, instance_id: str, region: str, backend_data: Optional[str] = None) -> None:
        shim = LocalShim._per_instance.pop(instance_id, None)
        if shim is not None:
            shim.stop()  # a per-instance agent goes with its instance; the shared one stays

    # instance volumes only: a "volume" is a directory under the server dir
    def create_volume(self, volume: Volume) -> VolumeProvisioningData:
        from dstack_amd.server import settings

        path = settings.SERVER_DIR_PATH / "volumes" / volume.name
        path.mkdir(parents=True, exist_ok=True)
        return VolumeProvisioningData(backend=BackendType.LOCAL, volume_id=str(path),
                                      size_gb=int(volume.configuration.size or 0), attachable=True)

    def register_volume(self, volume: Volume) -> VolumeProvisioningData:
        return VolumeProvisioningData(backend=BackendType.LOCAL, volume_id=volume.configuration.volume_id or "",
                                      size_gb=int(volume.configuration.size or 0))

    def delete_volume(self, volume: Volume) -> None:
        return None

    def attach_volume(self, volume, instance_id):
        from dstack_amd.core.models.volumes import VolumeAttachmentData

        return VolumeAttachmentData(device_name=None)

    def detach_volume(self, volume, instance_id, force=False):
        return None
