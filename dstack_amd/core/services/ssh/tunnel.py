"""SSH tunnels over the system ``ssh`` binary (reference: ``C/services/ssh/tunnel.py:61-279``,
``S/services/runner/ssh.py:22-86``).

The reference opens an ``ssh -f -N -L`` tunnel (a fork) for every runner/shim call, which is the
dominant per-call latency of its cold start.  Here a ``TunnelPool`` keeps one ControlMaster
connection per host and adds port forwards to it on demand (``ssh -O forward``), so after the
first call a runner/shim request costs one loopback HTTP round trip.
"""

from __future__ import annotations

import os
import socket
import subprocess
import tempfile
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from dstack_amd.core.errors import SSHError


def find_free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass(frozen=True)
class SSHTarget:
    hostname: str
    username: str
    port: int = 22
    proxy: Optional["SSHTarget"] = None


@dataclass
class _Master:
    target: SSHTarget
    control_path: str
    identity_file: str
    proc: Optional[subprocess.Popen] = None
    forwards: Dict[Tuple[str, int], int] = field(default_factory=dict)


def _base_opts(identity_file: str, port: int) -> List[str]:
    return [
        "-i", identity_file, "-p", str(port),
        "-o", "StrictHostKeyChecking=no", "-o", "UserKnownHostsFile=/dev/null", "-o", "LogLevel=ERROR",
        "-o", "ServerAliveInterval=30", "-o", "ServerAliveCountMax=4", "-o", "ConnectTimeout=10",
        "-o", "ExitOnForwardFailure=yes", "-o", "IdentitiesOnly=yes",
    ]


def _proxy_opts(target: SSHTarget, identity_file: str) -> List[str]:
    if target.proxy is None:
        return []
    p = target.proxy
    jump = (f"ssh -i {identity_file} -p {p.port} -o StrictHostKeyChecking=no -o UserKnownHostsFile=/dev/null "
            f"-W %h:%p {p.username}@{p.hostname}")
    return ["-o", f"ProxyCommand={jump}"]


class TunnelPool:
    def __init__(self, control_dir: Optional[str] = None):
        self._dir = control_dir or tempfile.mkdtemp(prefix="dstack-ssh-")
        self._masters: Dict[SSHTarget, _Master] = {}
        self._lock = threading.Lock()

    def _key_file(self, private_key: str) -> str:
        import hashlib

        h = hashlib.sha1(private_key.encode()).hexdigest()[:16]
        path = os.path.join(self._dir, f"key-{h}")
        if not os.path.exists(path):
            with open(path, "w") as f:
                f.write(private_key if private_key.endswith("\n") else private_key + "\n")
            os.chmod(path, 0o600)
        return path

    def _master(self, target: SSHTarget, private_key: str) -> _Master:
        with self._lock:
            m = self._masters.get(target)
            if m is not None and m.proc is not None and m.proc.poll() is None:
                return m
            ident = self._key_file(private_key)
            cp = os.path.join(self._dir, f"cm-{abs(hash(target)) % 10**10}")
            m = _Master(target=target, control_path=cp, identity_file=ident)
            cmd = ["ssh", "-N", "-M", "-S", cp, *_base_opts(ident, target.port), *_proxy_opts(target, ident),
                   f"{target.username}@{target.hostname}"]
            m.proc = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            deadline = time.monotonic() + 20
            while not os.path.exists(cp):
                if m.proc.poll() is not None:
                    err = m.proc.stderr.read().decode(errors="ignore") if m.proc.stderr else ""
                    raise SSHError(f"ssh to {target.hostname} failed: {err.strip()}")
                if time.monotonic() > deadline:
                    m.proc.kill()
                    raise SSHError(f"ssh to {target.hostname} timed out")
                time.sleep(0.02)
            self._masters[target] = m
            return m

    def forward(self, target: SSHTarget, private_key: str, remote_port: int, remote_host: str = "localhost") -> int:
        """Local port forwarding ``127.0.0.1:<local> -> <remote_host>:<remote_port>`` on ``target``."""
        m = self._master(target, private_key)
        key = (remote_host, remote_port)
        with self._lock:
            if key in m.forwards:
                return m.forwards[key]
            local = find_free_port()
            r = subprocess.run(["ssh", "-S", m.control_path, "-O", "forward", "-L",
                                f"127.0.0.1:{local}:{remote_host}:{remote_port}", f"{target.username}@{target.hostname}"],
                               capture_output=True, text=True, timeout=20)
            if r.returncode != 0:
                raise SSHError(f"ssh forward failed: {r.stderr.strip()}")
            m.forwards[key] = local
            return local

    def run(self, target: SSHTarget, private_key: str, command: str, timeout: float = 600, input: Optional[bytes] = None):
        """Run a command on the host over the master connection."""
        m = self._master(target, private_key)
        return subprocess.run(["ssh", "-S", m.control_path, f"{target.username}@{target.hostname}", command],
                              input=input, capture_output=True, timeout=timeout)

    def copy(self, target: SSHTarget, private_key: str, local_path: str, remote_path: str, timeout: float = 600):
        m = self._master(target, private_key)
        return subprocess.run(["scp", "-o", f"ControlPath={m.control_path}", "-P", str(target.port),
                               "-o", "StrictHostKeyChecking=no", "-o", "UserKnownHostsFile=/dev/null",
                               local_path, f"{target.username}@{target.hostname}:{remote_path}"],
                              capture_output=True, timeout=timeout)

    def close(self, target: SSHTarget):
        with self._lock:
            m = self._masters.pop(target, None)
        if m and m.proc:
            subprocess.run(["ssh", "-S", m.control_path, "-O", "exit", f"{target.username}@{target.hostname}"],
                           capture_output=True)
            m.proc.terminate()

    def close_all(self):
        for t in list(self._masters):
            self.close(t)


_pool: Optional[TunnelPool] = None


def get_tunnel_pool() -> TunnelPool:
    global _pool
    if _pool is None:
        _pool = TunnelPool()
    return _pool


@dataclass(frozen=True)
class IPSocket:
    host: str
    port: int

    def spec(self) -> str:
        host = f"[{self.host}]" if ":" in self.host else self.host  # IPv6 literals are bracketed
        return f"{host}:{self.port}"


@dataclass(frozen=True)
class UnixSocket:
    path: str

    def spec(self) -> str:
        return self.path


@dataclass(frozen=True)
class SocketPair:
    local: object  # IPSocket | UnixSocket
    remote: object


def ports_to_forwarded_sockets(ports: Dict[int, int], bind_local: str = "127.0.0.1") -> List[SocketPair]:
    """{remote port: local port} -> local-forward socket pairs bound on ``bind_local``."""
    return [SocketPair(local=IPSocket(bind_local, lp), remote=IPSocket("localhost", rp)) for rp, lp in ports.items()]


class SSHTunnel:
    """One ``ssh -N -f`` master with local (``-L``) and reverse (``-R``) forwards over TCP or unix
    sockets, addressed later through its control socket (check / exit / exec) -- the CLI's
    attach.  The identity is a key file path or the key's content (written to a private temp
    file); ``ssh_config_path`` None means ``-F none`` (the user's config is not consulted)."""

    def __init__(self, target: SSHTarget, identity_file: Optional[str] = None,
                 forwards: Optional[List[Tuple[int, str, int]]] = None, control_sock_path: Optional[str] = None,
                 identity_content: Optional[str] = None, options: Optional[Dict[str, str]] = None,
                 ssh_config_path: Optional[str] = None, forwarded_sockets: Optional[List[SocketPair]] = None,
                 reverse_forwarded_sockets: Optional[List[SocketPair]] = None, ssh_binary: str = "ssh"):
        self.target = target
        self.temp_dir = tempfile.TemporaryDirectory(prefix="dstack-tunnel-")
        if identity_content is not None:
            identity_file = os.path.join(self.temp_dir.name, "identity")
            with open(identity_file, "w") as f:
                f.write(identity_content)
            os.chmod(identity_file, 0o600)
        self.identity_file = identity_file
        self.forwarded_sockets = list(forwarded_sockets or []) + [
            SocketPair(IPSocket("127.0.0.1", local), IPSocket(host, remote)) for local, host, remote in (forwards or [])]
        self.reverse_forwarded_sockets = list(reverse_forwarded_sockets or [])
        self.control_sock_path = control_sock_path or os.path.join(self.temp_dir.name, "control.sock")
        self.options = dict(options) if options is not None else {
            "StrictHostKeyChecking": "no", "UserKnownHostsFile": "/dev/null", "LogLevel": "ERROR",
            "ServerAliveInterval": "30", "ExitOnForwardFailure": "yes", "IdentitiesOnly": "yes"}
        self.ssh_config_path = ssh_config_path
        self.ssh = ssh_binary

    @property
    def destination(self) -> str:
        return f"{self.target.username}@{self.target.hostname}"

    def open_command(self) -> List[str]:
        cmd = [self.ssh, "-F", self.ssh_config_path or "none"]
        if self.identity_file:
            cmd += ["-i", self.identity_file]
        cmd += ["-E", os.path.join(self.temp_dir.name, "tunnel.log"), "-N", "-f", "-o", "ControlMaster=auto",
                "-S", self.control_sock_path]
        if self.target.port and self.target.port != 22:
            cmd += ["-p", str(self.target.port)]
        for k, v in self.options.items():
            cmd += ["-o", f"{k}={v}"]
        if self.target.proxy is not None:
            p = self.target.proxy
            jump = [self.ssh] + (["-i", self.identity_file] if self.identity_file else []) + [
                "-W", "%h:%p", "-o", "StrictHostKeyChecking=no", "-o", "UserKnownHostsFile=/dev/null",
                "-p", str(p.port), f"{p.username}@{p.hostname}"]
            cmd += ["-o", "ProxyCommand=" + " ".join(jump)]
        for sp in self.forwarded_sockets:
            cmd += ["-L", f"{sp.local.spec()}:{sp.remote.spec()}"]
        for sp in self.reverse_forwarded_sockets:  # -R remote:local
            cmd += ["-R", f"{sp.remote.spec()}:{sp.local.spec()}"]
        cmd.append(self.destination)
        return cmd

    def check_command(self) -> List[str]:
        return [self.ssh, "-S", self.control_sock_path, "-O", "check", self.destination]

    def close_command(self) -> List[str]:
        return [self.ssh, "-S", self.control_sock_path, "-O", "exit", self.destination]

    def exec_command(self) -> List[str]:
        return [self.ssh, "-S", self.control_sock_path, self.destination]

    def open(self, timeout: float = 20):
        r = subprocess.run(self.open_command(), capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            log = os.path.join(self.temp_dir.name, "tunnel.log")
            detail = open(log).read().strip() if os.path.exists(log) else r.stderr.strip()
            raise SSHError(detail or f"ssh exited with {r.returncode}")

    def close(self):
        subprocess.run(self.close_command(), capture_output=True)

    def __enter__(self):
        self.open()
        return self

    def __exit__(self, *a):
        self.close()
