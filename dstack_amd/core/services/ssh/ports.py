"""Local port reservation for ``dstack attach`` (reference: ``core/services/ssh/ports.py:12-76``).

A port is held by a bound (unlistened) socket until the tunnel that will own it is about to start,
so two concurrent ``dstack apply`` calls cannot pick the same local port.
"""

from __future__ import annotations

import socket
from typing import Dict, Optional


class PortUsedError(Exception):
    pass


class PortsLock:
    def __init__(self, restrictions: Optional[Dict[int, int]] = None):
        """``restrictions``: remote port -> requested local port (0 = any free port)."""
        self.restrictions = dict(restrictions or {})
        self.sockets: Dict[int, socket.socket] = {}

    def acquire(self) -> "PortsLock":
        assigned = set()
        for remote, local in self.restrictions.items():
            if local:
                if local in assigned:
                    raise PortUsedError(f"Port {local} is requested twice")
                self.sockets[remote] = _bind(local)
                assigned.add(local)
        for remote, local in self.restrictions.items():
            if not local:
                self.sockets[remote] = _bind(remote) if _free(remote) and remote not in assigned else _bind(0)
                assigned.add(self.sockets[remote].getsockname()[1])
        return self

    def release(self) -> Dict[int, int]:
        mapping = self.dict()
        for s in self.sockets.values():
            s.close()
        self.sockets.clear()
        return mapping

    def dict(self) -> Dict[int, int]:
        return {r: s.getsockname()[1] for r, s in self.sockets.items()}


def _free(port: int) -> bool:
    try:
        _bind(port).close()
        return True
    except PortUsedError:
        return False


def _bind(port: int) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind(("127.0.0.1", port))
    except OSError as e:
        s.close()
        raise PortUsedError(f"Port {port} is already in use") from e
    return s
