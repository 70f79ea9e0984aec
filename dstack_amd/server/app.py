"""FastAPI application (reference: ``S/app.py:67-271``).

Lifespan: migrations -> encryption keys -> admin user + default project + ``config.yml`` -> local
backend shim -> reconcilers (event-driven scheduler) -> prints the admin token.
"""

from __future__ import annotations

import logging
import os
import time
from contextlib import asynccontextmanager
from typing import Optional

from fastapi import FastAPI, Request
from fastapi.exceptions import RequestValidationError
from fastapi.responses import JSONResponse

from dstack_amd import __version__
from dstack_amd.core.errors import (
    ForbiddenError,
    ResourceNotExistsError,
    ResourceBusyError,
    ServerClientError,
    UnauthorizedError,
)
from dstack_amd.server import settings
from dstack_amd.server.db import migrate, session_scope
from dstack_amd.server.utils.routers import check_client_server_compatibility

logger = logging.getLogger("dstack_amd.server")


def configure_logging(level: Optional[str] = None):
    lvl = getattr(logging, (level or settings.SERVER_LOG_LEVEL).upper(), logging.INFO)
    fmt = "%(asctime)s %(levelname)s %(name)s: %(message)s"
    if settings.SERVER_LOG_FORMAT == "json":
        fmt = '{"ts": "%(asctime)s", "level": "%(levelname)s", "logger": "%(name)s", "msg": "%(message)s"}'
    logging.basicConfig(level=getattr(logging, settings.SERVER_ROOT_LOG_LEVEL, logging.ERROR), format=fmt)
    logging.getLogger("dstack_amd").setLevel(lvl)
    logging.getLogger("httpx").setLevel(logging.WARNING)


def init_server_state(admin_token: Optional[str] = None):
    """Idempotent bootstrap shared by the app lifespan and tests."""
    from dstack_amd.server.services.config import ServerConfigManager
    from dstack_amd.server.services.pools import get_or_create_default_pool
    from dstack_amd.server.services.projects import get_or_create_default_project
    from dstack_amd.server.services.users import get_or_create_admin_user

    migrate()
    cm = ServerConfigManager()
    if not settings.SERVER_CONFIG_DISABLED:
        cm.load_config()
        cm.apply_encryption()
    with session_scope() as s:
        admin = get_or_create_admin_user(s, admin_token or settings.SERVER_ADMIN_TOKEN)
        project = get_or_create_default_project(s, admin, settings.DEFAULT_PROJECT_NAME)
        get_or_create_default_pool(s, project)
        cm.apply_config(s, admin)
        token = admin.token
    return token


def init_sentry():
    """Optional error/trace reporting (reference ``S/app.py:67-76``): active when
    ``DSTACK_SENTRY_DSN`` is set and the ``sentry_sdk`` package is installed."""
    if not settings.SENTRY_DSN:
        return False
    try:
        import sentry_sdk
    except ImportError:
        logger.warning("DSTACK_SENTRY_DSN is set but sentry_sdk is not installed")
        return False
    sentry_sdk.init(dsn=settings.SENTRY_DSN, traces_sample_rate=settings.SENTRY_TRACES_SAMPLE_RATE,
                    profiles_sample_rate=settings.SENTRY_PROFILES_SAMPLE_RATE,
                    environment=settings.SERVER_ENVIRONMENT, release=__version__)
    return True


def create_app(start_background: bool = True) -> FastAPI:
    @asynccontextmanager
    async def lifespan(app: FastAPI):
        from starlette.concurrency import run_in_threadpool

        token = await run_in_threadpool(init_server_state)
        app.state.admin_token = token
        if start_background:
            from dstack_amd.server.services.gateways import init_gateways

            try:
                await run_in_threadpool(init_gateways)
            except Exception:  # noqa: BLE001 - gateways must never keep the server from starting
                logger.exception("gateway init failed")
        sched = None
        if start_background and settings.SERVER_BACKGROUND_PROCESSING_ENABLED:
            from dstack_amd.server.background import start_background_tasks

            sched = start_background_tasks()
        url = settings.SERVER_URL
        print(f"The admin token is {token}", flush=True)
        print(f"The dstack-amd server {__version__} is running at {url}", flush=True)
        _write_client_config(url, token)
        yield
        if sched is not None:
            sched.shutdown()
        from dstack_amd.core.backends.local import LocalShim

        if LocalShim._instance is not None:
            LocalShim._instance.stop()
        from dstack_amd.server.services.gateways import LocalGatewayProcess

        LocalGatewayProcess.stop_all()

    init_sentry()
    app = FastAPI(title="dstack-amd", version=__version__, lifespan=lifespan, docs_url="/api/docs",
                  openapi_url="/api/openapi.json")
    register_routes(app)
    return app


def _write_client_config(url: str, token: str):
    """Make the local CLI usable right after `dstack server` (reference ``update_default_project``):
    the project becomes the CLI's default when the CLI has none yet; a different default project is
    replaced only after a confirmation on a terminal, or with ``DSTACK_UPDATE_DEFAULT_PROJECT``;
    ``DSTACK_DO_NOT_UPDATE_DEFAULT_PROJECT`` never writes."""
    if os.environ.get("DSTACK_SERVER_NO_CLIENT_CONFIG") or settings.DO_NOT_UPDATE_DEFAULT_PROJECT:
        return
    try:
        from dstack_amd.core.services.configs import ConfigManager

        cm = ConfigManager()
        current = cm.get_project_config()  # the CLI's default project
        if current is not None and (current.name, current.url, current.token) == (settings.DEFAULT_PROJECT_NAME, url,
                                                                                   token):
            return
        if current is not None and not settings.UPDATE_DEFAULT_PROJECT:
            import sys

            if not sys.stdin.isatty():
                logger.info("the CLI's default project is %s at %s; left as is (DSTACK_UPDATE_DEFAULT_PROJECT=1 "
                            "replaces it)", current.name, current.url)
                return
            from rich.prompt import Confirm

            if not Confirm.ask(f"Update the {settings.DEFAULT_PROJECT_NAME} project in the CLI config?"):
                return
        cm.configure_project(settings.DEFAULT_PROJECT_NAME, url, token, default=True)
        cm.save()
    except Exception as e:  # noqa: BLE001
        logger.debug("client config not written: %s", e)


def _error(status: int, msg: str, code: str) -> JSONResponse:
    return JSONResponse(status_code=status, content={"detail": [{"msg": msg, "code": code}]})


def register_routes(app: FastAPI):
    from dstack_amd.server.routers import core, proxy, runs

    for r in (core.server_router, core.users_router, core.projects_router, core.backends_router,
              core.project_backends_router, core.secrets_router, core.repos_router, runs.runs_root,
              runs.runs_router, runs.fleets_root, runs.fleets_router, runs.instances_root, runs.volumes_root,
              runs.volumes_router, runs.gateways_router, runs.logs_router, runs.metrics_router, runs.pools_root,
              runs.pool_router, runs.configs_router, proxy.router):
        app.include_router(r)

    @app.exception_handler(UnauthorizedError)
    async def _unauth(request: Request, exc: UnauthorizedError):
        return _error(401, exc.msg, exc.code)

    @app.exception_handler(ForbiddenError)
    async def _forbidden(request: Request, exc: ForbiddenError):
        return _error(403, exc.msg, exc.code)

    @app.exception_handler(ResourceNotExistsError)
    async def _notfound(request: Request, exc: ResourceNotExistsError):
        return _error(400, exc.msg, exc.code)

    @app.exception_handler(ResourceBusyError)
    async def _busy(request: Request, exc: ResourceBusyError):
        return _error(409, exc.msg, exc.code)

    @app.exception_handler(ServerClientError)
    async def _client_error(request: Request, exc: ServerClientError):
        return _error(400, exc.msg, exc.code)

    @app.exception_handler(RequestValidationError)
    async def _validation(request: Request, exc: RequestValidationError):
        return JSONResponse(status_code=422, content={"detail": jsonable_errors(exc.errors())})

    @app.middleware("http")
    async def log_request(request: Request, call_next):
        start = time.perf_counter()
        err = check_client_server_compatibility(request.headers.get("x-api-version"), _server_version())
        if err:
            return _error(400, err, "error")
        response = await call_next(request)
        logger.debug("%s %s %s %.1f ms", request.method, request.url.path, response.status_code,
                     (time.perf_counter() - start) * 1e3)
        return response

    @app.get("/healthcheck")
    def healthcheck():
        return {"status": "running"}

    from pathlib import Path

    from fastapi.responses import HTMLResponse

    ui_index = Path(__file__).parent / "ui" / "index.html"

    @app.get("/", include_in_schema=False)
    def ui():
        """Web UI (single page over the REST API)."""
        return HTMLResponse(ui_index.read_text() if ui_index.exists() else "<h3>dstack-amd</h3>")

    ui_assets = {p.name: p for p in (Path(__file__).parent / "ui" / "js").glob("*.js")}

    @app.get("/ui/js/{name}", include_in_schema=False)
    def ui_asset(name: str):
        """The UI's script modules (a fixed whitelist: the files shipped in ``server/ui/js``)."""
        from fastapi.responses import PlainTextResponse

        p = ui_assets.get(name)
        if p is None:
            return PlainTextResponse("not found", status_code=404)
        return PlainTextResponse(p.read_text(), media_type="text/javascript",
                                 headers={"Cache-Control": "no-cache"})

    @app.get("/metrics", include_in_schema=False)
    def prometheus_metrics():
        """Prometheus exposition (DSTACK_ENABLE_PROMETHEUS_METRICS=0 disables it)."""
        from fastapi.responses import PlainTextResponse

        if os.environ.get("DSTACK_ENABLE_PROMETHEUS_METRICS", "1") in ("0", "false"):
            return PlainTextResponse("", status_code=404)
        from dstack_amd.server.services.prometheus import render

        with session_scope() as s:
            return PlainTextResponse(render(s), media_type="text/plain; version=0.0.4")

    @app.get("/api/server/scheduler_stats")
    def scheduler_stats():
        from dstack_amd.server.background.scheduler import get_scheduler

        return get_scheduler().stats()


def jsonable_errors(errors):
    out = []
    for e in errors:
        out.append({k: (str(v) if k == "ctx" else v) for k, v in e.items() if k != "input"})
    return out


def _server_version() -> Optional[str]:
    """None for development builds (``0.0.x``): they accept every client."""
    return None if __version__.startswith("0.0") else __version__
