"""``dstack-gateway`` process (reference: ``P/gateway/main.py`` + systemd unit in
``gateway/src/dstack/gateway/resources/systemd``): control app on 127.0.0.1:8000 and, without
nginx, the built-in data plane on :80 (or ``--http-port``)."""

from __future__ import annotations

import argparse
import asyncio
import os
from pathlib import Path


def main(argv=None):
    ap = argparse.ArgumentParser("dstack-gateway")
    ap.add_argument("--state-dir", default=os.path.expanduser("~/dstack"))
    ap.add_argument("--control-port", type=int, default=8000)
    ap.add_argument("--http-port", type=int, default=80)
    ap.add_argument("--server-url", default=os.getenv("DSTACK_GATEWAY_SERVER_URL"))
    ap.add_argument("--identity-file", default=os.path.expanduser("~/.ssh/id_rsa"))
    ap.add_argument("--data-plane", choices=("auto", "nginx", "builtin"), default="auto")
    a = ap.parse_args(argv)
    import uvicorn

    from dstack_amd.proxy.gateway.app import Gateway, make_app, make_dataplane_app
    from dstack_amd.proxy.gateway.nginx import Nginx

    use_nginx = a.data_plane == "nginx" or (a.data_plane == "auto" and Nginx.available())
    nginx = Nginx(app_port=a.control_port, http_port=a.http_port) if use_nginx else None
    if nginx is not None:
        nginx.write_common()
    gw = Gateway(Path(a.state_dir), nginx, a.server_url,
                 a.identity_file if os.path.exists(a.identity_file) else None)
    control = uvicorn.Server(uvicorn.Config(make_app(gw), host="127.0.0.1", port=a.control_port, log_level="info"))
    servers = [control]
    if nginx is None:
        dp = make_dataplane_app(gw)
        dp.state.control_port = a.control_port
        servers.append(uvicorn.Server(uvicorn.Config(dp, host="0.0.0.0", port=a.http_port, log_level="warning")))

    async def serve():
        await asyncio.gather(*(s.serve() for s in servers))

    try:
        asyncio.run(serve())
    finally:
        gw.conns.close_all()


if __name__ == "__main__":
    main()
