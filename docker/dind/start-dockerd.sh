#!/bin/bash
# start dockerd in the background, then run the given command (the dstack-runner bootstrap)
set -e
dockerd-entrypoint.sh >/var/log/dockerd.log 2>&1 &
for i in $(seq 60); do docker info >/dev/null 2>&1 && break; sleep 1; done
exec "$@"
