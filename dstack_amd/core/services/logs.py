"""Client-side log rewriting (reference: ``src/dstack/_internal/core/services/logs.py``).

A job prints the URLs its servers listen on inside the container (``http://0.0.0.0:8000/...``).
``URLReplacer`` rewrites them, in the raw log bytes, into URLs the user can open: for an attached
task the forwarded local port on ``127.0.0.1`` (plus the app's query parameters, e.g. a Jupyter
token), for a service the service's public address (https default port omitted, the in-server
proxy's path prefix added).
"""

from __future__ import annotations

import re
from typing import Dict, List, Optional

from dstack_amd.core.models.runs import AppSpec


class URLReplacer:
    def __init__(self, ports: Dict[int, int], app_specs: List[AppSpec], hostname: str, secure: bool,
                 path_prefix: str = "", ip_address: Optional[str] = None):
        self.ports = {int(k): int(v) for k, v in ports.items()}
        self.apps = {a.port: a for a in app_specs}
        self.hostname = hostname
        self.secure = secure
        self.path_prefix = path_prefix.encode()
        hosts = [b"0.0.0.0", b"localhost", b"127.0.0.1"] + ([ip_address.encode()] if ip_address else [])
        self._re = re.compile(rb"(https?)://(" + b"|".join(re.escape(h) for h in hosts) +
                              rb")(?::(\d+))?(/[^\s\x1b\"'<>]*)?")

    def _sub(self, m: "re.Match[bytes]") -> bytes:
        scheme = m.group(1)
        port = int(m.group(3)) if m.group(3) else (443 if scheme == b"https" else 80)
        if port not in self.ports:
            return m.group(0)
        new_port = self.ports[port]
        path = m.group(4) or b""
        if self.path_prefix and not path.startswith(self.path_prefix.rstrip(b"/")):
            path = self.path_prefix.rstrip(b"/") + b"/" + path.lstrip(b"/")
        app = self.apps.get(port)
        if app is not None and app.url_query_params:
            q = "&".join(f"{k}={v}" for k, v in app.url_query_params.items()).encode()
            path = path + (b"&" if b"?" in path else b"?") + q
        out_scheme = b"https" if self.secure else b"http"
        default = 443 if self.secure else 80
        netloc = self.hostname.encode() + (b"" if new_port == default else b":%d" % new_port)
        return out_scheme + b"://" + netloc + path

    def __call__(self, chunk: bytes) -> bytes:
        return self._re.sub(self._sub, chunk)
