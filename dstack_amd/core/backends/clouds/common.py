"""Shared machinery for the cloud backends (reference: ``C/backends/base/compute.py:45-451`` and the
per-cloud ``compute.py`` files).

The reference drives each cloud through its Python SDK (boto3, azure-mgmt, google-cloud, oci,
kubernetes, ...).  None of those SDKs ship with this image, and they are not needed: every
backend here talks to the cloud's public REST API with ``httpx`` and signs requests itself
(AWS SigV4, OCI/GCP RSA-SHA256 via the system OpenSSL).  Each ``Compute`` accepts an injected
``httpx.Client`` so tests drive it against a mock transport.

``VMCompute`` is the common shape of the VM clouds: offers from the offline catalog (MI300X /
MI325X / MI355X first), ``create_instance`` boots a VM whose cloud-init installs ``dstack-shim``,
``update_provisioning_data`` polls until the VM has an address, ``terminate_instance`` deletes it.
"""

from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import json
import threading
import os
import subprocess
import tempfile
import time
import urllib.parse
from typing import Dict, List, Optional, Tuple

import httpx

from dstack_amd.core.backends.base import Compute, get_docker_commands, get_user_data
from dstack_amd.core.backends.catalog import CatalogRow, catalog_fetch_timeout, get_catalog_offers
from dstack_amd.core.errors import BackendAuthError, ComputeError, NoCapacityError
from dstack_amd.core.models.instances import (
    InstanceAvailability,
    InstanceConfiguration,
    InstanceOfferWithAvailability,
)
from dstack_amd.core.models.runs import JobProvisioningData, Requirements

DEFAULT_SHIM_URL = "https://dstack-amd-releases.s3.amazonaws.com/latest/dstack-shim-linux-amd64"
DEFAULT_RUNNER_URL = "https://dstack-amd-releases.s3.amazonaws.com/latest/dstack-runner-linux-amd64"


def agent_urls() -> Tuple[str, str]:
    """Where fresh hosts download the native agents (``DSTACK_{SHIM,RUNNER}_DOWNLOAD_URL``)."""
    return (os.getenv("DSTACK_SHIM_DOWNLOAD_URL", DEFAULT_SHIM_URL),
            os.getenv("DSTACK_RUNNER_DOWNLOAD_URL", DEFAULT_RUNNER_URL))


def cloud_init(instance_config: InstanceConfiguration, backend_commands: Optional[List[str]] = None) -> str:
    shim, runner = agent_urls()
    return get_user_data(instance_config.get_public_keys(), shim, runner, backend_commands)


def container_commands(authorized_keys: List[str]) -> List[str]:
    return get_docker_commands(authorized_keys, agent_urls()[1])


def check_response(r: httpx.Response, what: str) -> httpx.Response:
    if r.status_code in (401, 403):
        raise BackendAuthError(f"{what}: {r.status_code} {r.text[:300]}")
    if r.status_code == 409 or (r.status_code >= 400 and any(
            s in r.text.lower() for s in ("capacity", "insufficient", "out of stock", "not available", "quota"))):
        raise NoCapacityError(f"{what}: {r.status_code} {r.text[:300]}")
    if r.status_code >= 400:
        raise ComputeError(f"{what}: {r.status_code} {r.text[:500]}")
    return r


_catalog_fetch = threading.local()


def _catalog_timeout_hook(request: httpx.Request) -> None:
    """httpx request hook: inside a live catalog fetch (this thread), requests get the short catalog
    timeout instead of the client's launch-sized one."""
    t = getattr(_catalog_fetch, "timeout", None)
    if t:
        request.extensions["timeout"] = httpx.Timeout(t).as_dict()


def install_catalog_timeout(client: httpx.Client) -> httpx.Client:
    hooks = client.event_hooks.get("request", [])
    if _catalog_timeout_hook not in hooks:
        client.event_hooks = {**client.event_hooks, "request": [*hooks, _catalog_timeout_hook]}
    return client


class CatalogOffers:
    """``get_offers`` from the catalog layers (catalog.py): the backend's live listing when it has
    one (``_fetch_catalog``), else the offline catalog."""

    # ---- offers -------------------------------------------------------------------------------
    # disk sizes (GB) the cloud lets us choose at launch, for catalog rows without a fixed disk
    CONFIGURABLE_DISK: Tuple[float, Optional[float]] = (1.0, None)

    def get_offers(self, requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
        fetch = None
        if self.has_online_catalog():
            def fetch():
                _catalog_fetch.timeout = catalog_fetch_timeout()
                try:
                    return self._fetch_catalog()
                finally:
                    _catalog_fetch.timeout = None
        offers = get_catalog_offers(self.TYPE, self.regions(), requirements, self.CONFIGURABLE_DISK,
                                    extra_filter=self._offer_filter, fetch=fetch, cache_key=self.catalog_key())
        avail = self._availability()
        for o in offers:
            a = avail.get((o.instance.name, o.region)) if avail else None
            if a is not None:
                o.availability = a
        return offers

    def regions(self) -> Optional[List[str]]:
        """Configured region filter (``regions``; Azure's configs call them ``locations``)."""
        return self.config.get("regions") or self.config.get("locations")

    def has_online_catalog(self) -> bool:
        """True when the backend implements a live listing and it is not switched off
        (``offline_catalog: true`` in the backend config or ``DSTACK_CATALOG_OFFLINE_ONLY=1``)."""
        if self.config.get("offline_catalog") or os.getenv("DSTACK_CATALOG_OFFLINE_ONLY") == "1":
            return False
        return type(self)._fetch_catalog is not CatalogOffers._fetch_catalog

    def catalog_key(self) -> str:
        """Online-cache key: backend type + a fingerprint of the credentials / account settings."""
        ident = json.dumps([self.auth, self.config.get("project_id"), self.config.get("subscription_id")],
                           sort_keys=True, default=str)
        return f"{self.TYPE.value}:{hashlib.sha256(ident.encode()).hexdigest()[:16]}"

    def _fetch_catalog(self) -> List[CatalogRow]:
        """Live listing of the cloud's instance types (price + availability); see catalog.py."""
        raise NotImplementedError

    def _offer_filter(self, offer: InstanceOfferWithAvailability) -> bool:
        return True

    def check_credentials(self) -> None:
        """One cheap authenticated call; raises ``BackendAuthError`` when the cloud rejects the
        credentials (the server refuses to store such a backend).  Default: nothing to check."""
        return None

    def _availability(self) -> Dict[Tuple[str, str], InstanceAvailability]:
        """Optional extra stock overlay on top of the catalog rows."""
        return {}


class VMCompute(CatalogOffers, Compute):
    """Catalog offers + REST provisioning hooks (``_launch`` / ``_describe`` / ``_terminate``)."""

    SSH_USER = "ubuntu"
    DOCKERIZED = True

    def __init__(self, config: Dict, auth: Dict, client: Optional[httpx.Client] = None):
        super().__init__()
        self.config = config or {}
        self.auth = auth or {}
        self.http = install_catalog_timeout(client or httpx.Client(timeout=60))

    # ---- lifecycle ----------------------------------------------------------------------------
    def create_instance(self, instance_offer: InstanceOfferWithAvailability,
                        instance_config: InstanceConfiguration) -> JobProvisioningData:
        instance_id, hostname, backend_data = self._launch(instance_offer, instance_config)
        return JobProvisioningData(
            backend=self.TYPE, instance_type=instance_offer.instance, instance_id=instance_id, hostname=hostname,
            internal_ip=None, region=instance_offer.region, price=instance_offer.price,
            username=(backend_data or {}).get("ssh_user") or self.SSH_USER,  # a configured OS image's user
            ssh_port=22, dockerized=self.DOCKERIZED, backend_data=json.dumps(backend_data) if backend_data else None)

    def update_provisioning_data(self, provisioning_data: JobProvisioningData, project_ssh_public_key: str = "",
                                 project_ssh_private_key: str = "") -> None:
        if provisioning_data.hostname:
            return
        info = self._describe(provisioning_data.instance_id, provisioning_data.region,
                              json.loads(provisioning_data.backend_data or "{}"))
        if info.get("status") in ("failed", "terminated", "error"):
            raise ProvisioningFailed(f"{self.TYPE.value} instance {provisioning_data.instance_id}: {info}")
        if info.get("hostname"):
            provisioning_data.hostname = info["hostname"]
            provisioning_data.internal_ip = info.get("internal_ip")
            if info.get("ssh_port"):
                provisioning_data.ssh_port = int(info["ssh_port"])

    def terminate_instance(self, instance_id: str, region: str, backend_data: Optional[str] = None) -> None:
        self._terminate(instance_id, region, json.loads(backend_data or "{}"))

    # hooks
    def _launch(self, offer: InstanceOfferWithAvailability, cfg: InstanceConfiguration
                ) -> Tuple[str, Optional[str], Optional[dict]]:
        raise NotImplementedError

    def _describe(self, instance_id: str, region: str, backend_data: dict) -> dict:
        raise NotImplementedError

    def _terminate(self, instance_id: str, region: str, backend_data: dict) -> None:
        raise NotImplementedError


class ProvisioningFailed(ComputeError):
    pass


# ---------------------------------------------------------------------------------------------
# request signing
# ---------------------------------------------------------------------------------------------
def rsa_sha256_sign(private_key_pem: str, data: bytes, pss: bool = False) -> bytes:
    """RSA / SHA-256 signature with the system ``openssl`` (no crypto wheel needed): PKCS#1 v1.5, or
    PSS with a digest-length salt (JWT ``PS256``) when ``pss``."""
    with tempfile.NamedTemporaryFile("w", delete=False, suffix=".pem") as f:
        f.write(private_key_pem)
        key_path = f.name
    try:
        os.chmod(key_path, 0o600)
        cmd = ["openssl", "dgst", "-sha256", "-sign", key_path]
        if pss:
            cmd += ["-sigopt", "rsa_padding_mode:pss", "-sigopt", "rsa_pss_saltlen:-1"]
        r = subprocess.run(cmd, input=data, capture_output=True)
        if r.returncode != 0:
            raise BackendAuthError(f"openssl signing failed: {r.stderr.decode()[-300:]}")
        return r.stdout
    finally:
        os.unlink(key_path)


def ssh_key_fingerprint(public_key: str) -> str:
    """OpenSSH ``SHA256:`` fingerprint of a public key line (``type base64 [comment]``): clouds that
    store account-level keys under free-form names are matched on the key itself, never the name."""
    import hashlib

    parts = public_key.strip().split()
    blob = base64.b64decode(parts[1] if len(parts) > 1 else parts[0])
    return "SHA256:" + base64.b64encode(hashlib.sha256(blob).digest()).decode().rstrip("=")


def b64url(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def sigv4_headers(method: str, url: str, region: str, service: str, access_key: str, secret_key: str,
                  body: bytes = b"", session_token: Optional[str] = None, now: Optional[_dt.datetime] = None,
                  extra_headers: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """AWS Signature Version 4 for one request (query or JSON APIs)."""
    now = now or _dt.datetime.now(_dt.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    date = now.strftime("%Y%m%d")
    u = urllib.parse.urlsplit(url)
    payload_hash = hashlib.sha256(body).hexdigest()
    headers = {"host": u.netloc, "x-amz-date": amz_date, "x-amz-content-sha256": payload_hash}
    if session_token:
        headers["x-amz-security-token"] = session_token
    for k, v in (extra_headers or {}).items():
        headers[k.lower()] = v
    signed = sorted(headers)
    canonical_headers = "".join(f"{k}:{headers[k].strip()}\n" for k in signed)
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canonical_query = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                               for k, v in sorted(q))
    canonical = "\n".join([method, urllib.parse.quote(u.path or "/", safe="/-_.~"), canonical_query,
                           canonical_headers, ";".join(signed), payload_hash])
    scope = f"{date}/{region}/{service}/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canonical.encode()).hexdigest()])

    def _h(key: bytes, msg: str) -> bytes:
        return hmac.new(key, msg.encode(), hashlib.sha256).digest()

    k = _h(_h(_h(_h(("AWS4" + secret_key).encode(), date), region), service), "aws4_request")
    sig = hmac.new(k, to_sign.encode(), hashlib.sha256).hexdigest()
    out = {k2: v for k2, v in headers.items() if k2 != "host"}
    out["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, "
                            f"SignedHeaders={';'.join(signed)}, Signature={sig}")
    return out


class OAuthToken:
    """Cached bearer token from a client-credentials / JWT-bearer exchange."""

    def __init__(self, fetch):
        self._fetch = fetch
        self._token: Optional[str] = None
        self._exp = 0.0

    def get(self) -> str:
        if self._token is None or time.time() > self._exp - 60:
            tok, ttl = self._fetch()
            self._token, self._exp = tok, time.time() + float(ttl)
        return self._token
