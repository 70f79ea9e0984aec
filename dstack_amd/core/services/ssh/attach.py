"""``dstack attach``: local port forwards + an ``ssh <run-name>`` host entry (reference:
``core/services/ssh/attach.py:26-220``).

* local backend (process driver, host network): the job's ports already listen on this host, so
  only requested port *overrides* need a forward — done with an in-process TCP relay thread;
* remote hosts: one ``ssh -N -L ...`` with a ControlMaster socket per run, and Host blocks for
  ``<run>`` / ``<run>-host`` appended to ``~/.dstack/ssh/config`` (included from ``~/.ssh/config``
  by ``dstack config``) so users can ``ssh <run>``.
"""

from __future__ import annotations

import select
import socket
import subprocess
import threading
from pathlib import Path
from typing import Dict, List, Optional

from dstack_amd.core.errors import SSHError
from dstack_amd.core.services.ssh.ports import PortsLock


class _Relay:
    """Tiny TCP relay 127.0.0.1:local -> 127.0.0.1:remote (one thread per connection)."""

    def __init__(self, local_port: int, remote_port: int, bind: str = "127.0.0.1"):
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind((bind, local_port))
        self.srv.listen(64)
        self.remote_port = remote_port
        self._stop = False
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while not self._stop:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._pipe, args=(c,), daemon=True).start()

    def _pipe(self, c: socket.socket):
        try:
            u = socket.create_connection(("127.0.0.1", self.remote_port), timeout=10)
        except OSError:
            c.close()
            return
        socks = [c, u]
        try:
            while True:
                r, _, _ = select.select(socks, [], [], 60)
                if not r:
                    continue
                for s in r:
                    data = s.recv(65536)
                    if not data:
                        return
                    (u if s is c else c).sendall(data)
        except OSError:
            return
        finally:
            c.close()
            u.close()

    def close(self):
        self._stop = True
        self.srv.close()


def ssh_config_path() -> Path:
    from dstack_amd.core.services.configs import get_dstack_dir

    return get_dstack_dir() / "ssh" / "config"


def update_ssh_config(host: str, options: Optional[Dict[str, object]]):
    """Replace (or with ``options=None`` remove) the ``Host <host>`` block."""
    path = ssh_config_path()
    path.parent.mkdir(parents=True, exist_ok=True)
    lines = path.read_text().splitlines() if path.exists() else []
    out: List[str] = []
    skip = False
    for line in lines:
        if line.startswith("Host "):
            skip = line.split(None, 1)[1].strip() == host
        if not skip:
            out.append(line)
    if options is not None:
        out.append(f"Host {host}")
        out += [f"    {k} {v}" for k, v in options.items()]
    path.write_text("\n".join(out) + ("\n" if out else ""))


class RunAttach:
    def __init__(self, run, submission, identity_file: Optional[str], bind_address: str = "127.0.0.1",
                 ports_overrides: Optional[Dict[int, int]] = None):
        self.run_name = run.run_spec.run_name
        self.jpd = submission.job_provisioning_data
        self.jrd = submission.job_runtime_data
        conf = run.run_spec.configuration
        app_ports = [p.container_port for p in getattr(conf, "ports", []) or []]
        if getattr(conf, "type", None) == "service":
            app_ports.append(conf.port.container_port)
        if getattr(conf, "type", None) == "dev-environment":
            app_ports.append(getattr(conf, "ide_port", 0) or 0)
        self.remote_ports = [p for p in app_ports if p]
        self.overrides = ports_overrides or {}
        self.identity_file = identity_file
        self.bind = bind_address
        self.ports: Dict[int, int] = {}
        self._relays: List[_Relay] = []
        self._proc: Optional[subprocess.Popen] = None
        self._master = False  # a forwarding master (foreground or ControlPersist'ed) is up

    def _remote(self, p: int) -> int:
        if self.jrd is not None and self.jrd.ports:
            return int(self.jrd.ports.get(p, self.jrd.ports.get(str(p), p)))
        return p

    def open(self):
        local_backend = self.jpd is not None and self.jpd.backend.value == "local"
        if local_backend:
            for p in self.remote_ports:
                want = self.overrides.get(p)
                if want and want != self._remote(p):
                    self._relays.append(_Relay(want, self._remote(p), self.bind))
                    self.ports[p] = want
                else:
                    self.ports[p] = self._remote(p)
            return
        if self.identity_file is None:
            raise SSHError("attach needs an SSH identity file")
        lock = PortsLock({p: self.overrides.get(p, 0) for p in self.remote_ports}).acquire()
        mapping = lock.release()
        ctl = ssh_config_path().parent / f"{self.run_name}.control.sock"
        host_opts = {"HostName": self.jpd.hostname, "Port": self.jpd.ssh_port or 22, "User": self.jpd.username,
                     "IdentityFile": self.identity_file, "IdentitiesOnly": "yes", "StrictHostKeyChecking": "no",
                     "UserKnownHostsFile": "/dev/null"}
        update_ssh_config(f"{self.run_name}-host", host_opts)
        update_ssh_config(self.run_name, dict(host_opts, ControlPath=str(ctl)))
        cmd = ["ssh", "-F", str(ssh_config_path()), "-N", "-o", "ExitOnForwardFailure=yes", "-o", "ControlMaster=auto",
               "-o", f"ControlPath={ctl}", "-o", "ControlPersist=yes"]
        for remote, local in mapping.items():
            cmd += ["-L", f"{self.bind}:{local}:localhost:{self._remote(remote)}"]
        cmd.append(self.run_name)
        self._proc = self._connect(cmd)
        self._master = True
        self.ports = mapping

    def _connect(self, cmd: List[str]) -> Optional[subprocess.Popen]:
        """Start the forwarding master, retrying while the container's sshd is not up yet: the
        container bootstrap execs the runner first and brings sshd up in the background (possibly
        after installing it), so the first attach of a fresh job can find the port closed.  With
        ``ControlPersist`` the client backgrounds the master and exits 0 once connected; a refused
        or reset connection exits 255 and is retried with backoff until ``DSTACK_ATTACH_TIMEOUT``
        (default 180 s)."""
        import os
        import time

        deadline = time.monotonic() + float(os.getenv("DSTACK_ATTACH_TIMEOUT", 180))
        delay = 0.5
        while True:
            proc = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            try:
                rc = proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                return proc  # connected and holding the forwards in the foreground
            err = (proc.stderr.read() if proc.stderr else b"").decode(errors="replace").strip()
            if rc == 0:
                return None  # the persistent master runs in the background
            if time.monotonic() + delay > deadline:
                raise SSHError(f"cannot attach to {self.run_name}: ssh exited {rc}: {err[-500:]}")
            time.sleep(delay)
            delay = min(delay * 2, 5.0)

    def close(self):
        for r in self._relays:
            r.close()
        self._relays.clear()
        if self._proc is not None:
            self._proc.terminate()
            try:
                self._proc.wait(5)
            except subprocess.TimeoutExpired:
                self._proc.kill()
            self._proc = None
        if self._master:
            ctl = ssh_config_path().parent / f"{self.run_name}.control.sock"
            subprocess.run(["ssh", "-o", f"ControlPath={ctl}", "-O", "exit", self.run_name], capture_output=True,
                           timeout=10)
            self._master = False
            update_ssh_config(self.run_name, None)
            update_ssh_config(f"{self.run_name}-host", None)
