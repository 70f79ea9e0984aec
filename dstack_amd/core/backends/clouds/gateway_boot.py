"""Cloud-init for gateway VMs (reference: ``C/backends/base/compute.py:312-331,443-451``): nginx +
certbot + the ``dstack_amd.proxy.gateway`` app as a systemd service on 127.0.0.1:8000."""

from __future__ import annotations

import os

from dstack_amd.core.backends.base import json_quote
from dstack_amd.core.models.gateways import GatewayComputeConfiguration

GATEWAY_PACKAGE_URL = os.getenv("DSTACK_GATEWAY_PACKAGE_URL",
                                "https://dstack-amd-releases.s3.amazonaws.com/latest/dstack_amd-gateway.tar.gz")

SYSTEMD_UNIT = """[Unit]
Description=dstack-amd gateway
After=network.target nginx.service

[Service]
User=ubuntu
WorkingDirectory=/home/ubuntu
ExecStart=/home/ubuntu/venv/bin/python -m dstack_amd.proxy.gateway.main --data-plane nginx
Restart=always

[Install]
WantedBy=multi-user.target
"""


def gateway_commands(conf: GatewayComputeConfiguration) -> list:
    return [
        "apt-get update -qq && DEBIAN_FRONTEND=noninteractive apt-get install -yqq nginx certbot "
        "python3-certbot-nginx python3-venv",
        "python3 -m venv /home/ubuntu/venv",
        f"curl -fsSL '{GATEWAY_PACKAGE_URL}' | tar -xz -C /home/ubuntu",
        "/home/ubuntu/venv/bin/pip install -q fastapi uvicorn httpx jinja2 pydantic",
        "chown -R ubuntu:ubuntu /home/ubuntu",
        "echo 'ubuntu ALL=(ALL) NOPASSWD: /usr/sbin/nginx, /usr/bin/systemctl reload nginx, /usr/bin/certbot' "
        "> /etc/sudoers.d/dstack-gateway",
        f"printf %s {json_quote(SYSTEMD_UNIT)} > /etc/systemd/system/dstack-gateway.service",
        "systemctl daemon-reload && systemctl enable --now dstack-gateway",
    ]


def gateway_cloud_init(conf: GatewayComputeConfiguration) -> str:
    runcmd = "\n".join(f"  - {json_quote(c)}" for c in gateway_commands(conf))
    return f"#cloud-config\nssh_authorized_keys:\n  - {conf.ssh_key_pub.strip()}\nruncmd:\n{runcmd}\n"
