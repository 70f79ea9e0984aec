"""Client/server version compatibility (reference ``server/utils/routers.py:105-137``)."""

from __future__ import annotations

from typing import Optional

from packaging import version


def check_client_server_compatibility(client_version: Optional[str], server_version: Optional[str]) -> Optional[str]:
    """Error message when a client may not talk to this server, else None.

    A client is accepted unless it is a newer minor (or major) release than the server: patch
    releases stay compatible both ways and the server keeps serving older clients. ``latest`` (the
    web UI, development builds) skips the check, as does a server or client that sends no version."""
    if client_version is None or server_version is None or client_version == "latest":
        return None
    try:
        client = version.parse(client_version)
    except version.InvalidVersion:
        return "Bad API version specified"
    server = version.parse(server_version)
    if client > server and (client.major > server.major or client.minor > server.minor):
        return (f"The client/CLI version ({client_version}) is incompatible with the server version "
                f"({server_version}); use a client of version {server.major}.{server.minor} or older")
    return None
