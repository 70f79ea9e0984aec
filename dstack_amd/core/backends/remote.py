"""``remote`` backend: on-prem SSH fleets (reference: ``C/backends/remote/provisioning.py:50-296``).

Deployment of a host (``deploy_ssh_instance``) over the system ssh/scp (paramiko is not
available): append the project key to authorized_keys, copy ``dstack-shim``/``dstack-runner``
(+ ``dstack-probe``), write ``shim.env``, start the shim (systemd unit when systemd is there,
otherwise nohup), read ``host_info`` (amdsmi topology) and health-check the shim.  The host's
resources become the instance type; ``blocks: auto`` later splits it along xGMI sub-meshes.
"""

from __future__ import annotations

import json
import shlex
import time
from typing import Dict, List, Optional, Tuple

from dstack_amd.core.backends.base import DSTACK_SHIM_HTTP_PORT, Compute
from dstack_amd.core.errors import ProvisioningError, SSHError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import (
    Disk,
    Gpu,
    HostTopology,
    InstanceOfferWithAvailability,
    InstanceType,
    RemoteConnectionInfo,
    Resources,
)
from dstack_amd.core.models.runs import Requirements
from dstack_amd.core.services.ssh.tunnel import SSHTarget, get_tunnel_pool
from dstack_amd import native_bin

REMOTE_SHIM_DIR = "~/.dstack-shim"
SHIM_UNIT = """[Unit]
Description=dstack-shim (MI355X orchestrator host agent)
After=network-online.target

[Service]
Type=simple
User=root
EnvironmentFile={dir}/shim.env
ExecStart={dir}/dstack-shim --service --shim-home {dir} --runner-binary-path {dir}/dstack-runner {probe}
Restart=always
RestartSec=2

[Install]
WantedBy=multi-user.target
"""


class RemoteCompute(Compute):
    TYPE = BackendType.REMOTE

    def get_offers(self, requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
        return []  # SSH fleet capacity is the pool instances themselves

    def terminate_instance(self, instance_id: str, region: str, backend_data: Optional[str] = None) -> None:
        return None  # on-prem hosts are released, not destroyed (shim stopped by process_instances)


def host_info_to_instance_type(host_info: dict) -> Tuple[InstanceType, HostTopology]:
    topo_raw = host_info.get("topology") or {}
    topo = HostTopology(
        gpus=[{"index": g.get("index", i), "name": g.get("name") or "AMD GPU", "vendor": g.get("vendor") or "amd",
               "memory_mib": int(g.get("memory_mib") or 0), "bdf": g.get("bdf"),
               "render_node": g.get("render_node"), "arch": g.get("arch"), "serial": g.get("serial")}
              for i, g in enumerate(topo_raw.get("gpus", []))],
        xgmi=topo_raw.get("xgmi") or [],
        numa={int(k): int(v) for k, v in (topo_raw.get("numa") or {}).items()},
        nics=topo_raw.get("nics") or [],
    )
    gpus = [Gpu(name=g.name, memory_mib=g.memory_mib, vendor=g.vendor) for g in topo.gpus]
    res = Resources(cpus=int(host_info.get("cpus") or 1), memory_mib=int((host_info.get("memory") or 0) / 2**20),
                    gpus=gpus, spot=False, disk=Disk(size_mib=int((host_info.get("disk_size") or 0) / 2**20)))
    name = f"{len(gpus)}x{gpus[0].name}" if gpus else "ssh"
    return InstanceType(name=name, resources=res), topo


def deploy_ssh_instance(rci: RemoteConnectionInfo, project_public_key: str, private_key: str,
                        timeout: float = 20 * 60) -> dict:
    """Install and start the shim on an SSH host; returns host_info."""
    target = SSHTarget(rci.host, rci.ssh_user, rci.port)
    pool = get_tunnel_pool()
    shim, runner, probe = native_bin.shim_path(), native_bin.runner_path(), native_bin.probe_path()
    if not shim or not runner:
        raise ProvisioningError("native agents are not built")
    r = pool.run(target, private_key, f"mkdir -p {REMOTE_SHIM_DIR} && uname -m && (command -v systemctl || true)")
    if r.returncode != 0:
        raise SSHError(r.stderr.decode(errors="ignore"))
    has_systemd = b"systemctl" in r.stdout
    # authorized_keys: make the project key valid for this host (provisioning.py:56-96)
    key = project_public_key.strip()
    pool.run(target, private_key,
             f"mkdir -p ~/.ssh && touch ~/.ssh/authorized_keys && grep -qF {shlex.quote(key)} ~/.ssh/authorized_keys "
             f"|| echo {shlex.quote(key)} >> ~/.ssh/authorized_keys")
    for src, name in ((shim, "dstack-shim"), (runner, "dstack-runner"), (probe, "dstack-probe")):
        if src:
            cp = pool.copy(target, private_key, src, f".dstack-shim/{name}.new")
            if cp.returncode != 0:
                raise ProvisioningError(f"copy {name} failed: {cp.stderr.decode(errors='ignore')}")
            pool.run(target, private_key, f"mv -f {REMOTE_SHIM_DIR}/{name}.new {REMOTE_SHIM_DIR}/{name} && "
                                          f"chmod +x {REMOTE_SHIM_DIR}/{name}")
    env = dict(rci.env.items()) if len(rci.env) else {}
    env.setdefault("DSTACK_SHIM_HTTP_PORT", str(DSTACK_SHIM_HTTP_PORT))
    env_lines = "".join(f"{k}={v}\n" for k, v in env.items())
    pool.run(target, private_key, f"cat > {REMOTE_SHIM_DIR}/shim.env", input=env_lines.encode())
    probe_flag = f"--probe-binary $HOME/.dstack-shim/dstack-probe" if probe else ""
    if has_systemd and rci.ssh_user == "root":
        unit = SHIM_UNIT.format(dir="/root/.dstack-shim", probe=probe_flag.replace("$HOME", "/root"))
        pool.run(target, private_key, "cat > /etc/systemd/system/dstack-shim.service", input=unit.encode())
        pool.run(target, private_key, "systemctl daemon-reload && systemctl enable dstack-shim && "
                                      "systemctl restart dstack-shim")
    else:
        # restart the previous shim by its pid file (never by process name: other users' or
        # other installations' agents may run on the same host)
        pool.run(target, private_key,
                 f"cd {REMOTE_SHIM_DIR} && rm -f host_info.json && "
                 f"([ -f shim.pid ] && kill $(cat shim.pid) 2>/dev/null; true) && set -a && . ./shim.env && set +a && "
                 f"(nohup ./dstack-shim --service --shim-home $HOME/.dstack-shim --runner-binary-path "
                 f"$HOME/.dstack-shim/dstack-runner {probe_flag} > shim.log 2>&1 < /dev/null & echo $! > shim.pid)")
    deadline = time.monotonic() + min(timeout, 180)
    host_info = None
    while time.monotonic() < deadline:  # poll host_info.json (provisioning.py:175-202)
        r = pool.run(target, private_key, f"cat {REMOTE_SHIM_DIR}/host_info.json 2>/dev/null || true")
        out = r.stdout.decode(errors="ignore").strip()
        if out:
            try:
                host_info = json.loads(out)
                break
            except ValueError:
                pass
        time.sleep(1)
    if host_info is None:
        raise ProvisioningError("shim did not report host_info")
    return host_info


def remote_backend_data(shim_port: int = DSTACK_SHIM_HTTP_PORT, direct: bool = False) -> str:
    return json.dumps({"shim_port": shim_port, "direct": direct})


def auto_blocks(n_gpus: int, cpus: int) -> int:
    """``blocks: auto`` = as many blocks as the host can be cut into: one per GPU (each block
    needs at least one CPU, so never more than the CPUs); a CPU-only host, one per CPU (reference
    ``process_instances`` block rules)."""
    if n_gpus:
        return max(1, min(n_gpus, cpus) if cpus else n_gpus)
    return max(1, cpus)


def split_blocks(topo: HostTopology, blocks, cpus: int = 0) -> int:
    """Blocks of a host: ``auto`` per ``auto_blocks``; an explicit count must divide the GPUs
    (and CPUs) evenly.  The xGMI-aware allocator hands out fully-connected GPU subsets (MI355X
    nodes are all-to-all xGMI, so any subset works)."""
    n = len(topo.gpus)
    if blocks == "auto":
        return auto_blocks(n, cpus)
    blocks = int(blocks)
    if n and n % blocks != 0:
        raise ProvisioningError(f"{n} GPUs cannot be split into {blocks} blocks")
    if cpus and cpus % blocks != 0:
        raise ProvisioningError(f"{cpus} CPUs cannot be split into {blocks} blocks")
    return blocks
