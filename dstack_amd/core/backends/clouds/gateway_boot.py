"""Cloud-init for gateway VMs (reference: ``C/backends/base/compute.py:312-331,443-451``): nginx +
certbot + the versioned ``dstack_amd.proxy.gateway`` app as a systemd service on 127.0.0.1:8000,
installed into a blue/green slot by ``update.sh`` (``dstack_amd/proxy/gateway/packaging.py``)."""

from __future__ import annotations

from dstack_amd.core.backends.base import json_quote
from dstack_amd.core.models.gateways import GatewayComputeConfiguration
from dstack_amd.proxy.gateway.packaging import SYSTEMD_UNIT, install_commands, package_url  # noqa: F401


def gateway_commands(conf: GatewayComputeConfiguration) -> list:
    return install_commands(package_url())


def gateway_cloud_init(conf: GatewayComputeConfiguration) -> str:
    runcmd = "\n".join(f"  - {json_quote(c)}" for c in gateway_commands(conf))
    return f"#cloud-config\nssh_authorized_keys:\n  - {conf.ssh_key_pub.strip()}\nruncmd:\n{runcmd}\n"
