"""Server settings from the environment (reference: ``S/settings.py:1-73``)."""

from __future__ import annotations

import os
from pathlib import Path


def _env_bool(name: str, default: bool = False) -> bool:
    v = os.getenv(name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


DSTACK_DIR_PATH = Path(os.getenv("DSTACK_DIR", Path.home() / ".dstack"))
SERVER_DIR_PATH = Path(os.getenv("DSTACK_SERVER_DIR", DSTACK_DIR_PATH / "server"))
SERVER_CONFIG_FILE_PATH = SERVER_DIR_PATH / "config.yml"
SERVER_DATA_DIR_PATH = SERVER_DIR_PATH / "data"

DATABASE_URL = os.getenv("DSTACK_DATABASE_URL", f"sqlite:///{SERVER_DATA_DIR_PATH}/sqlite.db")
DB_POOL_SIZE = int(os.getenv("DSTACK_DB_POOL_SIZE", "20"))
DB_MAX_OVERFLOW = int(os.getenv("DSTACK_DB_MAX_OVERFLOW", "20"))

SERVER_HOST = os.getenv("DSTACK_SERVER_HOST", "127.0.0.1")
SERVER_PORT = int(os.getenv("DSTACK_SERVER_PORT", "3000"))
SERVER_URL = os.getenv("DSTACK_SERVER_URL", f"http://{SERVER_HOST}:{SERVER_PORT}")
SERVER_ADMIN_TOKEN = os.getenv("DSTACK_SERVER_ADMIN_TOKEN")
SERVER_LOG_LEVEL = os.getenv("DSTACK_SERVER_LOG_LEVEL", "INFO").upper()
SERVER_LOG_FORMAT = os.getenv("DSTACK_SERVER_LOG_FORMAT", "standard")  # standard | json | rich
# level of the root logger (third-party libraries); the server's own loggers use SERVER_LOG_LEVEL
SERVER_ROOT_LOG_LEVEL = os.getenv("DSTACK_SERVER_ROOT_LOG_LEVEL", "ERROR").upper()
SERVER_UVICORN_LOG_LEVEL = os.getenv("DSTACK_SERVER_UVICORN_LOG_LEVEL", "ERROR").lower()
SERVER_ENVIRONMENT = os.getenv("DSTACK_SERVER_ENVIRONMENT", "dev")  # reported to Sentry
# ignore ~/.dstack/server/config.yml entirely (neither read, applied nor created)
SERVER_CONFIG_DISABLED = os.getenv("DSTACK_SERVER_CONFIG_DISABLED") is not None
SQL_ECHO_ENABLED = os.getenv("DSTACK_SQL_ECHO_ENABLED") is not None

# in-server service proxy: how long one upstream request may take (LLM generations are long)
PROXY_UPSTREAM_TIMEOUT = float(os.getenv("DSTACK_PROXY_UPSTREAM_TIMEOUT", "600"))

SERVER_METRICS_TTL_SECONDS = int(os.getenv("DSTACK_SERVER_METRICS_TTL_SECONDS", "3600"))
SERVER_METRICS_COLLECT_INTERVAL = float(os.getenv("DSTACK_SERVER_METRICS_COLLECT_INTERVAL", "10"))
SERVER_BACKGROUND_PROCESSING_ENABLED = not _env_bool("DSTACK_SERVER_BACKGROUND_PROCESSING_DISABLED")
# Event-driven scheduling: background tasks are woken on state changes; the interval is only the
# fallback poll. Set to 0 to reproduce the reference's pure-polling behaviour.
SERVER_EVENT_DRIVEN = not _env_bool("DSTACK_SERVER_POLLING_ONLY")
# server start: do not update the app on running gateways (reference DSTACK_SKIP_GATEWAY_UPDATE)
SKIP_GATEWAY_UPDATE = _env_bool("DSTACK_SKIP_GATEWAY_UPDATE")

SERVER_CLOUDWATCH_LOG_GROUP = os.getenv("DSTACK_SERVER_CLOUDWATCH_LOG_GROUP")
# code blobs in S3 instead of the database (DSTACK_SERVER_S3_BUCKET is the older name here)
SERVER_S3_BUCKET = os.getenv("DSTACK_SERVER_BUCKET") or os.getenv("DSTACK_SERVER_S3_BUCKET")
SERVER_BUCKET_REGION = os.getenv("DSTACK_SERVER_BUCKET_REGION") or os.getenv("DSTACK_SERVER_S3_BUCKET_REGION")
SENTRY_DSN = os.getenv("DSTACK_SENTRY_DSN")
SENTRY_TRACES_SAMPLE_RATE = float(os.getenv("DSTACK_SENTRY_TRACES_SAMPLE_RATE", "0.1"))
SENTRY_PROFILES_SAMPLE_RATE = float(os.getenv("DSTACK_SENTRY_PROFILES_SAMPLE_RATE", "0"))

# backends may not use ambient (instance-role / environment) credentials: `creds: {type: default}`
DEFAULT_CREDS_DISABLED = os.getenv("DSTACK_DEFAULT_CREDS_DISABLED") is not None
# projects a new non-admin user may own
USER_PROJECT_DEFAULT_QUOTA = int(os.getenv("DSTACK_USER_PROJECT_DEFAULT_QUOTA", "10"))
# services must run behind a gateway (no in-server proxy)
FORBID_SERVICES_WITHOUT_GATEWAY = os.getenv("DSTACK_FORBID_SERVICES_WITHOUT_GATEWAY") is not None
# run every job container in bridge networking, also on hosts the job has to itself
FORCE_BRIDGE_NETWORK = _env_bool("DSTACK_FORCE_BRIDGE_NETWORK")
# server start: write the default project into the CLI config (~/.dstack/config.yml) always /
# never; by default only when the CLI config has no default project yet or points to this server
UPDATE_DEFAULT_PROJECT = os.getenv("DSTACK_UPDATE_DEFAULT_PROJECT") is not None
DO_NOT_UPDATE_DEFAULT_PROJECT = os.getenv("DSTACK_DO_NOT_UPDATE_DEFAULT_PROJECT") is not None

DEFAULT_PROJECT_NAME = "main"
LOCAL_BACKEND_ENABLED = _env_bool("DSTACK_LOCAL_BACKEND_ENABLED", True)
# where the local backend finds the native agents
SHIM_BINARY_PATH = os.getenv("DSTACK_SHIM_BINARY_PATH")
RUNNER_BINARY_PATH = os.getenv("DSTACK_RUNNER_BINARY_PATH")
RUNNER_DOWNLOAD_URL = os.getenv("DSTACK_RUNNER_DOWNLOAD_URL")
SHIM_DOWNLOAD_URL = os.getenv("DSTACK_SHIM_DOWNLOAD_URL")

SERVICE_CLIENT_MAX_BODY_SIZE = int(os.getenv("DSTACK_DEFAULT_SERVICE_CLIENT_MAX_BODY_SIZE")
                                   or os.getenv("DSTACK_SERVICE_CLIENT_MAX_BODY_SIZE") or 64 * 1024 * 1024)
ACME_SERVER = os.getenv("DSTACK_ACME_SERVER")
ACME_EAB_KID = os.getenv("DSTACK_ACME_EAB_KID")
ACME_EAB_HMAC_KEY = os.getenv("DSTACK_ACME_EAB_HMAC_KEY")

MAX_OFFERS_TRIED = int(os.getenv("DSTACK_SERVER_MAX_OFFERS_TRIED", "15"))
MAX_PLAN_OFFERS = 50
DEFAULT_RUNNER_TIMEOUT = 600


# identity of this server process among replicas sharing one database (leases such as the SSH-fleet
# deploy lease record it); fresh per process unless pinned
SERVER_REPLICA_ID = os.getenv("DSTACK_SERVER_REPLICA_ID") or __import__("uuid").uuid4().hex
