"""Run a throwaway dstack-amd server in a subprocess (used by the e2e tests and the cold-start
bench): temp ``DSTACK_DIR``, random admin token, free port, local backend, native agents."""

from __future__ import annotations

import os
import secrets
import shutil
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path
from typing import Dict, Optional

import httpx

REPO_ROOT = Path(__file__).resolve().parents[2]


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ServerProcess:
    def __init__(self, env: Optional[Dict[str, str]] = None, keep_dir: bool = False, log_level: str = "info"):
        self.dir = tempfile.mkdtemp(prefix="dstack-amd-")
        self.port = free_port()
        self.token = secrets.token_hex(16)
        self.url = f"http://127.0.0.1:{self.port}"
        self.extra_env = env or {}
        self.keep_dir = keep_dir
        self.log_level = log_level
        self.proc: Optional[subprocess.Popen] = None
        self.log_path = os.path.join(self.dir, "server.log")

    def start(self, timeout: float = 120.0) -> "ServerProcess":
        env = dict(os.environ)
        env.update({
            "DSTACK_DIR": os.path.join(self.dir, "home"), "DSTACK_SERVER_NO_CLIENT_CONFIG": "1",
            "PYTHONPATH": str(REPO_ROOT) + os.pathsep + env.get("PYTHONPATH", ""),
        })
        env.update(self.extra_env)
        self._log = open(self.log_path, "w")
        self.proc = subprocess.Popen(
            [sys.executable, "-m", "dstack_amd.server.main", "--port", str(self.port), "--token", self.token,
             "--log-level", self.log_level], env=env, stdout=self._log, stderr=subprocess.STDOUT,
            start_new_session=True)
        deadline = time.time() + timeout
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"server exited early:\n{self.log()}")
            try:
                if httpx.get(self.url + "/healthcheck", timeout=1).status_code == 200:
                    return self
            except httpx.HTTPError:
                pass
            time.sleep(0.1)
        self.stop()
        raise RuntimeError(f"server did not come up:\n{self.log()}")

    def log(self) -> str:
        try:
            return Path(self.log_path).read_text()[-8000:]
        except OSError:
            return ""

    def client(self):
        from dstack_amd.api import Client
        from dstack_amd.api.server import APIClient

        return Client(APIClient(self.url, self.token), "main")

    def stop(self):
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(15)
            except subprocess.TimeoutExpired:
                os.killpg(self.proc.pid, 9)
                self.proc.wait(5)
        self.proc = None
        if not self.keep_dir:
            shutil.rmtree(self.dir, ignore_errors=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()


def fake_amd_sysfs(root, n_gpus: int = 8, product: str = "AMD Instinct MI355X", vram_gib: int = 288,
                   xgmi: bool = True) -> str:
    """Build a fake ``/sys`` + ``/dev/dri`` tree of ``n_gpus`` AMD GPUs under ``root`` for the native
    agents' sysfs discovery (``DSTACK_SYSFS_ROOT``, ``native/common/amdgpu.cpp``): render nodes with
    vendor/product/VRAM, one PCI device per GPU, and a KFD topology whose io_links (type 11 = xGMI)
    fully connect the GPUs, as on an 8xMI355X OAM board.  Returns ``root`` as a string."""
    root = Path(root)
    nodes = root / "sys" / "class" / "kfd" / "kfd" / "topology" / "nodes"
    cpu = nodes / "0"
    cpu.mkdir(parents=True, exist_ok=True)
    (cpu / "gpu_id").write_text("0\n")
    (cpu / "properties").write_text("cpu_cores_count 8\nsimd_count 0\n")
    (root / "dev" / "dri").mkdir(parents=True, exist_ok=True)
    for i in range(n_gpus):
        bus = 0x05 + 0x10 * i
        bdf = f"0000:{bus:02x}:00.0"
        render = 128 + i
        dev = root / "sys" / "devices" / "pci0000:00" / bdf
        dev.mkdir(parents=True, exist_ok=True)
        (dev / "vendor").write_text("0x1002\n")
        (dev / "product_name").write_text(product + "\n")
        (dev / "mem_info_vram_total").write_text(str(vram_gib << 30) + "\n")
        (dev / "numa_node").write_text(f"{0 if i < n_gpus // 2 or n_gpus == 1 else 1}\n")
        drm = root / "sys" / "class" / "drm" / f"renderD{render}"
        drm.mkdir(parents=True, exist_ok=True)
        if not (drm / "device").exists():
            os.symlink(dev, drm / "device")
        (root / "dev" / "dri" / f"renderD{render}").write_text("")
        node = nodes / str(i + 1)
        (node / "io_links").mkdir(parents=True, exist_ok=True)
        (node / "gpu_id").write_text(f"{1000 + i}\n")
        (node / "properties").write_text(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        links = [0] + ([j + 1 for j in range(n_gpus) if j != i] if xgmi else [])
        for k, to in enumerate(links):
            ld = node / "io_links" / str(k)
            ld.mkdir(exist_ok=True)
            kind = 2 if to == 0 else 11  # PCIe to the CPU node, xGMI to every peer
            (ld / "properties").write_text(f"type {kind}\nnode_from {i + 1}\nnode_to {to}\nweight 15\n")
    return str(root)
