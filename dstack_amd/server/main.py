"""``dstack server`` entry point (reference: ``cli/commands/server.py:14-86`` +
``S/main.py``): uvicorn on one worker — all concurrency lives in the thread-pool handlers and the
event-driven scheduler threads, so one process owns the SQLite writer."""

from __future__ import annotations

import argparse
import os


def run(host: str = "127.0.0.1", port: int = 3000, log_level: str = "info", token: str | None = None):
    os.environ["DSTACK_SERVER_HOST"] = host
    os.environ["DSTACK_SERVER_PORT"] = str(port)
    os.environ.setdefault("DSTACK_SERVER_URL", f"http://{host}:{port}")
    if token:
        os.environ["DSTACK_SERVER_ADMIN_TOKEN"] = token
    import uvicorn

    from dstack_amd.server.app import configure_logging, create_app

    from dstack_amd.server import settings

    configure_logging(log_level)
    uvicorn.run(create_app(), host=host, port=port, log_level=settings.SERVER_UVICORN_LOG_LEVEL, access_log=False,
                timeout_graceful_shutdown=5)


def main(argv=None):
    ap = argparse.ArgumentParser("dstack-amd-server")
    ap.add_argument("--host", default=os.getenv("DSTACK_SERVER_HOST", "127.0.0.1"))
    ap.add_argument("--port", type=int, default=int(os.getenv("DSTACK_SERVER_PORT", "3000")))
    ap.add_argument("--log-level", default=os.getenv("DSTACK_SERVER_LOG_LEVEL", "info"))
    ap.add_argument("--token", default=os.getenv("DSTACK_SERVER_ADMIN_TOKEN"))
    a = ap.parse_args(argv)
    run(a.host, a.port, a.log_level, a.token)


if __name__ == "__main__":
    main()
