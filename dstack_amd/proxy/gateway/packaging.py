"""Versioned gateway package and blue/green updates (reference: the ``dstack-gateway`` wheel,
``gateway/src/dstack/gateway/resources/systemd/*`` and ``update.sh``; server side
``S/services/gateways/__init__.py:356-430``).

A gateway host keeps two source slots, ``~/dstack/blue`` and ``~/dstack/green``, and a symlink
``~/dstack/current`` to the live one; the systemd unit runs the app from ``current`` with one
shared venv for the third-party dependencies.  ``update.sh <package> <version>``:

1. unpacks the versioned package (``dstack_amd-gateway-<version>.tar.gz``: ``dstack_amd/proxy``
   and ``VERSION``) into the idle slot and checks its ``VERSION``;
2. switches ``current`` atomically (``ln -sfn`` + ``mv -T``) and restarts the service;
3. waits until ``/api/healthcheck`` reports the new version, else switches back to the previous
   slot, restarts it and exits 1 — a broken release never stays live.

The server pushes its own copy of ``update.sh`` before running it, so the update logic itself is
always the server's version.
"""

from __future__ import annotations

import io
import os
import tarfile
from typing import List, Optional

from dstack_amd import __version__

PACKAGE_NAME = "dstack_amd-gateway-{version}.tar.gz"
DEFAULT_PACKAGE_URL = "https://dstack-amd-releases.s3.amazonaws.com/{version}/" + PACKAGE_NAME
REQUIREMENTS = ["fastapi", "uvicorn", "httpx", "jinja2", "pydantic"]
GATEWAY_ROOT = "/home/ubuntu/dstack"

UPDATE_SH = r"""#!/bin/sh
# blue/green update of the dstack-amd gateway app
# usage: update.sh <package url or path> <version>
set -u
PKG="$1"
VERSION="$2"
ROOT="${DSTACK_GATEWAY_ROOT:-$HOME/dstack}"
PORT="${DSTACK_GATEWAY_PORT:-8000}"
RESTART="${DSTACK_GATEWAY_RESTART:-}"
if [ -z "$RESTART" ]; then
  # containers (no systemd) ship their own restart script next to the slots
  if [ -x "$ROOT/restart" ]; then RESTART="$ROOT/restart"; else RESTART="sudo systemctl restart dstack-gateway"; fi
fi
cur=$(readlink "$ROOT/current" 2>/dev/null || true)
case "$(basename "${cur:-none}")" in
  blue) next=green ;;
  *) next=blue ;;
esac
slot="$ROOT/$next"
rm -rf "$slot.tmp" && mkdir -p "$slot.tmp/src" || exit 1
case "$PKG" in
  http://*|https://*) curl -fsSL "$PKG" -o "$slot.tmp/pkg.tar.gz" || { echo "download failed: $PKG"; exit 1; } ;;
  *) cp "$PKG" "$slot.tmp/pkg.tar.gz" || { echo "no package: $PKG"; exit 1; } ;;
esac
tar -xzf "$slot.tmp/pkg.tar.gz" -C "$slot.tmp/src" || { echo "bad package"; exit 1; }
got=$(cat "$slot.tmp/src/VERSION" 2>/dev/null || true)
if [ "$got" != "$VERSION" ]; then echo "package version '$got' != '$VERSION'"; exit 1; fi
if [ -z "${DSTACK_GATEWAY_SKIP_PIP:-}" ] && [ -f "$slot.tmp/src/requirements.txt" ]; then
  "$ROOT/venv/bin/pip" install -q -r "$slot.tmp/src/requirements.txt" || { echo "pip install failed"; exit 1; }
fi
rm -rf "$slot" && mv "$slot.tmp" "$slot" || exit 1
switch() { ln -sfn "$1" "$ROOT/current.new" && mv -Tf "$ROOT/current.new" "$ROOT/current"; }
switch "$slot" || exit 1
$RESTART
i=0
while [ "$i" -lt "${DSTACK_GATEWAY_HEALTH_TRIES:-30}" ]; do
  if curl -fsS "http://127.0.0.1:$PORT/api/healthcheck" 2>/dev/null | grep -q "\"version\": *\"$VERSION\""; then
    echo "Update successfully completed"
    exit 0
  fi
  i=$((i + 1))
  sleep "${DSTACK_GATEWAY_HEALTH_SLEEP:-1}"
done
echo "version $VERSION did not become healthy; rolling back to ${cur:-nothing}"
if [ -n "$cur" ]; then
  switch "$cur"
  $RESTART
fi
exit 1
"""

SYSTEMD_UNIT = f"""[Unit]
Description=dstack-amd gateway
After=network.target nginx.service

[Service]
User=ubuntu
WorkingDirectory=/home/ubuntu
Environment=PYTHONPATH={GATEWAY_ROOT}/current/src
ExecStart={GATEWAY_ROOT}/venv/bin/python -m dstack_amd.proxy.gateway.main --data-plane nginx
Restart=always

[Install]
WantedBy=multi-user.target
"""


def package_url(version: str = __version__) -> str:
    """Where gateways fetch release ``version`` (``DSTACK_GATEWAY_PACKAGE_URL`` may hold a
    ``{version}`` placeholder, or a plain URL/path used as is)."""
    tpl = os.getenv("DSTACK_GATEWAY_PACKAGE_URL", DEFAULT_PACKAGE_URL)
    return tpl.format(version=version) if "{version}" in tpl else tpl


def _repo_root() -> str:
    return os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def build_package(out_dir: str, version: str = __version__) -> str:
    """Write ``dstack_amd-gateway-<version>.tar.gz``: the ``dstack_amd`` package root module, the
    ``dstack_amd/proxy`` subpackage (gateway app, registry, nginx, stats, model proxy), ``VERSION``
    and ``requirements.txt``.  Deterministic (sorted members, zeroed mtimes/owners), so the same
    source tree always gives the same bytes."""
    root = _repo_root()
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, PACKAGE_NAME.format(version=version))
    members: List[str] = [os.path.join("dstack_amd", "__init__.py")]
    for dirpath, dirnames, filenames in os.walk(os.path.join(root, "dstack_amd", "proxy")):
        dirnames[:] = sorted(d for d in dirnames if d != "__pycache__")
        for f in sorted(filenames):
            if f.endswith((".py", ".jinja2", ".conf")):
                members.append(os.path.relpath(os.path.join(dirpath, f), root))

    def _info(name: str, size: int) -> tarfile.TarInfo:
        ti = tarfile.TarInfo(name)
        ti.size, ti.mtime, ti.mode, ti.uid, ti.gid, ti.uname, ti.gname = size, 0, 0o644, 0, 0, "", ""
        return ti

    import gzip

    with open(path, "wb") as raw, gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as gz, \
            tarfile.open(fileobj=gz, mode="w") as tar:
        for rel in sorted(members):
            with open(os.path.join(root, rel), "rb") as f:
                data = f.read()
            tar.addfile(_info(rel, len(data)), io.BytesIO(data))
        for name, text in (("VERSION", version), ("requirements.txt", "\n".join(REQUIREMENTS) + "\n")):
            data = text.encode()
            tar.addfile(_info(name, len(data)), io.BytesIO(data))
    return path


def write_file_command(content: str, path: str, mode: Optional[str] = None) -> str:
    """A shell command that writes ``content`` to ``path`` byte for byte.  base64 keeps every ``$``,
    quote and newline of a script literal through cloud-init YAML, ``sh -c`` and SSH alike."""
    import base64

    b64 = base64.b64encode(content.encode()).decode()
    cmd = f"echo '{b64}' | base64 -d > {path}"
    return cmd + (f" && chmod {mode} {path}" if mode else "")


def install_commands(url: Optional[str] = None, version: str = __version__) -> List[str]:
    """First install on a fresh gateway VM (cloud-init, as root): shared venv, update script,
    systemd unit, then ``update.sh`` installs the release into the first slot and starts it."""
    url = url or package_url(version)
    r = GATEWAY_ROOT
    return [
        "apt-get update -qq && DEBIAN_FRONTEND=noninteractive apt-get install -yqq nginx certbot "
        "python3-certbot-nginx python3-venv curl",
        f"mkdir -p {r} && python3 -m venv {r}/venv",
        f"{r}/venv/bin/pip install -q " + " ".join(REQUIREMENTS),
        write_file_command(UPDATE_SH, f"{r}/update.sh"),
        "chown -R ubuntu:ubuntu /home/ubuntu",
        "echo 'ubuntu ALL=(ALL) NOPASSWD: /usr/sbin/nginx, /usr/bin/systemctl reload nginx, "
        "/usr/bin/systemctl restart dstack-gateway, /usr/bin/certbot' > /etc/sudoers.d/dstack-gateway",
        write_file_command(SYSTEMD_UNIT, "/etc/systemd/system/dstack-gateway.service"),
        "systemctl daemon-reload && systemctl enable dstack-gateway",
        f"sudo -u ubuntu env HOME=/home/ubuntu DSTACK_GATEWAY_SKIP_PIP=1 sh {r}/update.sh '{url}' '{version}'",
    ]


RESTART_SH = """#!/bin/sh
# (re)start the gateway app from the live slot: containers have no systemd
ROOT="${DSTACK_GATEWAY_ROOT:-$HOME/dstack}"
if [ -f "$ROOT/app.pid" ]; then kill "$(cat "$ROOT/app.pid")" 2>/dev/null; sleep 1; fi
PYTHONPATH="$ROOT/current/src" nohup "$ROOT/venv/bin/python" -m dstack_amd.proxy.gateway.main --data-plane nginx \\
  > "$ROOT/app.log" 2>&1 &
echo $! > "$ROOT/app.pid"
"""


def container_commands(ssh_key_pub: str, url: Optional[str] = None, version: str = __version__) -> List[str]:
    """Gateway in a plain ``ubuntu:22.04`` container (Kubernetes pod): sshd for the server's
    tunnel, nginx, the shared venv, the release installed by ``update.sh`` and started by the
    ``restart`` script; sshd stays in the foreground as the container's main process."""
    import shlex

    url = url or package_url(version)
    r = "/root/dstack"
    return [
        "export DEBIAN_FRONTEND=noninteractive",
        "apt-get update -qq && apt-get install -yqq openssh-server nginx certbot python3-certbot-nginx "
        "python3-venv curl",
        f"mkdir -p /root/.ssh /run/sshd {r} && chmod 700 /root/.ssh",
        f"printf '%s\\n' {shlex.quote(ssh_key_pub.strip())} >> /root/.ssh/authorized_keys",
        "chmod 600 /root/.ssh/authorized_keys && nginx",
        f"python3 -m venv {r}/venv && {r}/venv/bin/pip install -q " + " ".join(REQUIREMENTS),
        write_file_command(UPDATE_SH, f"{r}/update.sh"),
        write_file_command(RESTART_SH, f"{r}/restart", "+x"),
        f"cd /root && DSTACK_GATEWAY_SKIP_PIP=1 sh {r}/update.sh '{url}' '{version}'",
        "exec /usr/sbin/sshd -D",
    ]


def remote_update_command(url: str, version: str) -> str:
    """What the server runs over SSH (after pushing ``UPDATE_SH`` to ``dstack/update.sh``); a
    private copy keeps a running update from being overwritten by the next push."""
    return ("cp dstack/update.sh dstack/_update.sh && sh dstack/_update.sh "
            f"'{url}' '{version}'; rc=$?; rm -f dstack/_update.sh; exit $rc")
