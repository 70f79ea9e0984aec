"""Nginx site manager for the gateway data plane (reference: ``P/gateway/services/nginx.py:56-180``,
templates ``P/gateway/resources/nginx/*.jinja2``).

One site per service domain (``upstream`` of replica sockets/addresses + optional
``auth_request`` to the gateway app) and one per model entrypoint (``gateway.<domain>`` proxying
the OpenAI API to the gateway app).  Every change is written, validated with ``nginx -t`` and
reloaded; a failing config is rolled back to the previous file.  HTTPS certificates are obtained
with certbot (ACME server / EAB credentials optional).
"""

from __future__ import annotations

import logging
import os
import shutil
import subprocess
from pathlib import Path
from typing import Optional

import jinja2

from dstack_amd.proxy.gateway.registry import Entrypoint, Service
from dstack_amd.proxy.gateway.stats import LOG_FORMAT

logger = logging.getLogger(__name__)

SERVICE_TEMPLATE = """\
{% if upstreams %}upstream dstack_{{ name }} {
{% for u in upstreams %}    server {{ u }};
{% endfor %}    keepalive 64;
}
{% endif %}server {
    server_name {{ domain }};
    access_log {{ access_log }} dstack_stat;
    client_max_body_size {{ client_max_body_size }};
    listen {{ http_port }};
{% if https %}    listen {{ https_port }} ssl;
    ssl_certificate {{ certs_dir }}/{{ domain }}/fullchain.pem;
    ssl_certificate_key {{ certs_dir }}/{{ domain }}/privkey.pem;
    set $force_https 1;
    if ($scheme = "https") { set $force_https 0; }
    if ($remote_addr = 127.0.0.1) { set $force_https 0; }
    if ($force_https) { return 301 https://$host$request_uri; }
{% endif %}
    location / {
{% if auth %}        auth_request /_dstack_auth;
{% endif %}{% if upstreams %}        proxy_pass http://dstack_{{ name }};
        proxy_http_version 1.1;
        proxy_set_header Upgrade $http_upgrade;
        proxy_set_header Connection $connection_upgrade;
        proxy_set_header Host $host;
        proxy_set_header X-Real-IP $remote_addr;
        proxy_read_timeout 300s;
        proxy_buffering off;
{% else %}        return 503;
{% endif %}    }
{% if auth %}    location = /_dstack_auth {
        internal;
        proxy_pass http://127.0.0.1:{{ app_port }}/api/auth/{{ project }};
        proxy_pass_request_body off;
        proxy_set_header Content-Length "";
        proxy_set_header Authorization $http_authorization;
    }
{% endif %}}
"""

ENTRYPOINT_TEMPLATE = """\
server {
    server_name {{ domain }};
    access_log {{ access_log }} dstack_stat;
    listen {{ http_port }};
{% if https %}    listen {{ https_port }} ssl;
    ssl_certificate {{ certs_dir }}/{{ domain }}/fullchain.pem;
    ssl_certificate_key {{ certs_dir }}/{{ domain }}/privkey.pem;
{% endif %}    location / {
        proxy_pass http://127.0.0.1:{{ app_port }}/api/models/{{ project }}/;
        proxy_http_version 1.1;
        proxy_set_header Host $host;
        proxy_buffering off;
        proxy_read_timeout 300s;
    }
}
"""

COMMON_CONF = f"""\
log_format dstack_stat '{LOG_FORMAT}';
map $http_upgrade $connection_upgrade {{ default upgrade; '' close; }}
"""


class NginxError(RuntimeError):
    pass


class Nginx:
    def __init__(self, conf_dir: str = "/etc/nginx/sites-enabled", access_log: str = "/var/log/nginx/dstack.access.log",
                 app_port: int = 8000, http_port: int = 80, https_port: int = 443, reload_cmd=None,
                 test_cmd=None, certbot_cmd=None, certs_dir: str = "/etc/letsencrypt/live"):
        self.conf_dir = Path(conf_dir)
        self.access_log = access_log
        self.app_port = app_port
        self.http_port, self.https_port = http_port, https_port
        self.reload_cmd = reload_cmd or ["sudo", "systemctl", "reload", "nginx"]
        self.test_cmd = test_cmd or ["sudo", "nginx", "-t"]
        self.certbot_cmd = certbot_cmd or ["sudo", "certbot"]
        self.certs_dir = certs_dir
        self._env = jinja2.Environment(trim_blocks=False, keep_trailing_newline=True)

    @staticmethod
    def available() -> bool:
        return shutil.which("nginx") is not None

    def write_common(self):
        self._write("00-dstack-common.conf", COMMON_CONF)

    def render_service(self, svc: Service) -> str:
        ups = [r.upstream() for r in svc.replicas.values()]
        name = f"{svc.project}_{svc.run_name}".replace("-", "_")
        return self._env.from_string(SERVICE_TEMPLATE).render(
            name=name, upstreams=ups, domain=svc.domain, access_log=self.access_log,
            client_max_body_size=svc.client_max_body_size, https=svc.https, auth=svc.auth, project=svc.project,
            app_port=self.app_port, http_port=self.http_port, https_port=self.https_port, certs_dir=self.certs_dir)

    def render_entrypoint(self, ep: Entrypoint) -> str:
        return self._env.from_string(ENTRYPOINT_TEMPLATE).render(
            domain=ep.domain, access_log=self.access_log, https=ep.https, project=ep.project,
            app_port=self.app_port, http_port=self.http_port, https_port=self.https_port, certs_dir=self.certs_dir)

    def site_name(self, domain: str) -> str:
        return f"{self.http_port}-{domain}.conf"

    def apply_service(self, svc: Service):
        if svc.https:
            self.obtain_certificate(svc.domain)
        self._write(self.site_name(svc.domain), self.render_service(svc))

    def apply_entrypoint(self, ep: Entrypoint):
        if ep.https:
            self.obtain_certificate(ep.domain)
        self._write(self.site_name(ep.domain), self.render_entrypoint(ep))

    def remove(self, domain: str):
        p = self.conf_dir / self.site_name(domain)
        if p.exists():
            p.unlink()
            self._reload()

    def _write(self, name: str, text: str):
        self.conf_dir.mkdir(parents=True, exist_ok=True)
        path = self.conf_dir / name
        old: Optional[str] = path.read_text() if path.exists() else None
        if old == text:
            return
        path.write_text(text)
        try:
            self._run(self.test_cmd)
            self._reload()
        except NginxError:
            if old is None:
                path.unlink()
            else:
                path.write_text(old)
            raise

    def _reload(self):
        self._run(self.reload_cmd)

    @staticmethod
    def _run(cmd):
        if not cmd:
            return
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise NginxError(f"{' '.join(cmd)} failed: {r.stderr.strip()[-500:]}")

    def obtain_certificate(self, domain: str, acme_server: Optional[str] = None, eab_kid: Optional[str] = None,
                           eab_hmac_key: Optional[str] = None):
        if os.path.exists(f"{self.certs_dir}/{domain}/fullchain.pem"):
            return
        cmd = [*self.certbot_cmd, "certonly", "--non-interactive", "--agree-tos", "--register-unsafely-without-email",
               "--nginx", "--domain", domain]
        acme_server = acme_server or os.getenv("DSTACK_ACME_SERVER")
        if acme_server:
            cmd += ["--server", acme_server]
        eab_kid = eab_kid or os.getenv("DSTACK_ACME_EAB_KID")
        eab_hmac_key = eab_hmac_key or os.getenv("DSTACK_ACME_EAB_HMAC_KEY")
        if eab_kid and eab_hmac_key:
            cmd += ["--eab-kid", eab_kid, "--eab-hmac-key", eab_hmac_key]
        self._run(cmd)
