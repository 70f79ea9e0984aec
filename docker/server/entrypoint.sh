#!/bin/bash
# `docker run -p 3000:3000 -v ~/.dstack/server:/root/.dstack/server dstack-amd-server`
set -e
exec python -m dstack_amd.cli.main server --host "${DSTACK_SERVER_HOST:-0.0.0.0}" --port "${DSTACK_SERVER_PORT:-3000}" \
  ${DSTACK_SERVER_ADMIN_TOKEN:+--token "$DSTACK_SERVER_ADMIN_TOKEN"} "$@"
