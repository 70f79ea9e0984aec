"""OpenSSH client helpers (reference: ``src/dstack/_internal/utils/ssh.py``)."""

from __future__ import annotations

import re
import subprocess

REQUIRED_SSH_VERSION = (8, 4)  # ControlMaster + StreamLocalBindUnlink + ProxyJump behaviour the CLI relies on


def check_required_ssh_version(required=REQUIRED_SSH_VERSION) -> bool:
    """True when the local ``ssh`` is OpenSSH >= ``required`` (``ssh -V`` prints to stderr, the
    Windows build to stdout); False when it is older, not OpenSSH, or cannot be run."""
    try:
        r = subprocess.run(["ssh", "-V"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return False
    text = f"{r.stderr or ''} {r.stdout or ''}"
    m = re.search(r"OpenSSH(?:_for_Windows)?_(\d+)\.(\d+)", text)
    if m is None:
        return False
    return (int(m.group(1)), int(m.group(2))) >= tuple(required)


def get_ssh_config(host: str, path: str = "~/.ssh/config") -> dict:
    """The options ``~/.ssh/config`` gives ``host`` (lower-cased keys, first match wins as in
    ssh(1); ``Host`` patterns with ``*``/``?`` and ``!`` negation).  Missing file -> {}."""
    import fnmatch
    import os

    try:
        with open(os.path.expanduser(path)) as f:
            lines = f.read().splitlines()
    except OSError:
        return {}
    out: dict = {}
    active = True  # options before the first Host apply to every host
    for raw in lines:
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        key, _, value = line.replace("=", " ", 1).partition(" ")
        key, value = key.lower(), value.strip().strip('"')
        if key == "host":
            pats = value.split()
            neg = any(p.startswith("!") and fnmatch.fnmatch(host, p[1:]) for p in pats)
            active = not neg and any(not p.startswith("!") and fnmatch.fnmatch(host, p) for p in pats)
            continue
        if key == "match":
            active = False  # Match blocks are not evaluated here
            continue
        if active and key not in out:
            out[key] = value
    return out


from dataclasses import dataclass  # noqa: E402
from pathlib import Path  # noqa: E402
from typing import Tuple  # noqa: E402


@dataclass(frozen=True)
class SSHClientInfo:
    """What the local OpenSSH client can do (reference ``core/services/ssh/client.py``): the
    Windows port has no control sockets, so no multiplexing and no ``-f`` background mode; the
    MSYS2 build (Git for Windows) has control sockets but cannot multiplex."""

    path: Path
    version: str
    version_tuple: Tuple[int, ...]
    for_windows: bool
    supports_control_socket: bool
    supports_multiplexing: bool
    supports_background_mode: bool

    @classmethod
    def from_raw_version(cls, raw: str, path: Path, windows_host: bool = None) -> "SSHClientInfo":
        import sys

        m = re.match(r"OpenSSH_(for_Windows_)?(\d+\.\d+\S*?)[, ]", raw.strip() + " ")
        if m is None:
            raise ValueError(f"not an OpenSSH version string: {raw!r}")
        for_windows = bool(m.group(1))
        version = m.group(2)
        vt = tuple(int(x) for x in re.match(r"(\d+)\.(\d+)", version).groups())
        on_windows = sys.platform == "win32" if windows_host is None else windows_host
        return cls(path=path, version=version, version_tuple=vt, for_windows=for_windows,
                   supports_control_socket=not for_windows, supports_multiplexing=not (for_windows or on_windows),
                   supports_background_mode=not for_windows)
