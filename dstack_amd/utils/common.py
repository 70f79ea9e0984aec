"""Small shared helpers (reference: ``src/dstack/_internal/utils/common.py``,
``random_names.py``, ``crypto.py``, ``network.py``)."""

from __future__ import annotations

import hashlib
import ipaddress
import os
import random
import re
import secrets
import subprocess
import tempfile
from datetime import datetime, timedelta, timezone
from typing import Iterable, List, Optional, Tuple, TypeVar

T = TypeVar("T")


def get_current_datetime() -> datetime:
    """Naive UTC 'now' (the DB stores naive UTC)."""
    return datetime.now(timezone.utc).replace(tzinfo=None)


def to_aware(dt: Optional[datetime]) -> Optional[datetime]:
    if dt is None:
        return None
    return dt if dt.tzinfo else dt.replace(tzinfo=timezone.utc)


def pretty_date(dt: Optional[datetime], now: Optional[datetime] = None) -> str:
    """``now``, ``30 sec ago``, ``1 min ago`` / ``45 mins ago``, ``1 hour ago`` / ``5 hours ago``,
    ``yesterday``, ``5 days ago``, ``3 weeks ago``, ``3 months ago``, ``1 year ago``; a time in the
    future is ``""`` (reference ``utils/common.py`` ``pretty_date``)."""
    if dt is None:
        return "-"
    now = to_aware(now) if now is not None else datetime.now(timezone.utc)
    diff = now - to_aware(dt)
    s, days = int(diff.total_seconds()), diff.days
    if days < 0:
        return ""
    if days == 0:
        if s < 10:
            return "now"
        if s < 60:
            return f"{s} sec ago"
        if s < 3600:
            m = s // 60
            return f"{m} min{'s' if m > 1 else ''} ago"
        h = s // 3600
        return f"{h} hour{'s' if h > 1 else ''} ago"
    if days == 1:
        return "yesterday"
    if days < 7:
        return f"{days} days ago"
    for n, unit in ((365, "year"), (30, "month"), (7, "week")):
        if days >= n:
            k = days // n
            return f"{k} {unit}{'s' if k > 1 else ''} ago"
    return f"{days} days ago"


def local_time(dt: datetime) -> str:
    """``HH:MM`` of ``dt`` (naive values are taken as local time)."""
    return dt.strftime("%H:%M")


_MEMORY_UNITS = {"K": 2**10, "M": 2**20, "G": 2**30, "T": 2**40, "P": 2**50}


def parse_memory(memory: str, as_untis: str = "M") -> float:
    """A Kubernetes-style quantity (``1024Ki``, ``2Gi``, ``512M``) in ``as_untis`` (K|M|G|T)."""
    m = re.fullmatch(r"\s*([0-9.]+)\s*([KMGTP])?(i)?[Bb]?\s*", memory)
    if m is None:
        raise ValueError(f"cannot parse memory quantity {memory!r}")
    n = float(m.group(1))
    if m.group(2):
        n *= _MEMORY_UNITS[m.group(2)] if m.group(3) else 1000 ** ("KMGTP".index(m.group(2)) + 1)
    return n / _MEMORY_UNITS[as_untis.upper()[0]]


def split_chunks(iterable: Iterable[T], chunk_size: int) -> Iterable[List[T]]:
    """Consecutive lists of at most ``chunk_size`` items (any iterable, generators included)."""
    if chunk_size < 1:
        raise ValueError(f"chunk_size must be positive, got {chunk_size}")
    chunk: List[T] = []
    for x in iterable:
        chunk.append(x)
        if len(chunk) == chunk_size:
            yield chunk
            chunk = []
    if chunk:
        yield chunk


def concat_url_path(a, b):
    """Join two URL path parts with exactly one ``/`` between them (str or bytes; inner ``//``
    runs of the parts are kept)."""
    sep = b"/" if isinstance(a, bytes) else "/"
    if not b:
        return a
    a2 = a[:-1] if a.endswith(sep) else a
    b2 = b[1:] if b.startswith(sep) else b
    return a2 + sep + b2


def make_proxy_url(server_url: str, proxy_url: str) -> str:
    """Absolute URL of a service / model endpoint: absolute proxy URLs (gateways) as they are,
    in-server proxy paths appended to the server URL (keeping its path prefix)."""
    if "://" in proxy_url:
        return proxy_url
    return concat_url_path(server_url.rstrip("/"), proxy_url)


def format_pretty_duration(seconds: int) -> str:
    if seconds == 0:
        return "0s"
    out = []
    for unit, n in (("d", 86400), ("h", 3600), ("m", 60), ("s", 1)):
        if seconds >= n:
            out.append(f"{seconds // n}{unit}")
            seconds %= n
    return "".join(out)


_ADJ = ["amber", "bold", "brave", "calm", "clever", "cool", "crisp", "eager", "fast", "fierce", "gentle", "giant",
        "happy", "keen", "lively", "lucky", "mighty", "nimble", "noble", "proud", "quick", "quiet", "rapid", "sharp",
        "shiny", "silent", "smooth", "steady", "swift", "tidy", "vivid", "wise"]
_NOUN = ["aardvark", "badger", "bison", "cobra", "condor", "crane", "dingo", "eagle", "falcon", "ferret", "gecko",
         "heron", "ibis", "jaguar", "koala", "lemur", "lynx", "marmot", "moose", "narwhal", "ocelot", "otter", "panda",
         "puma", "quokka", "raven", "salmon", "tapir", "toucan", "walrus", "wombat", "yak", "zebra"]


def generate_name() -> str:
    return f"{random.choice(_ADJ)}-{random.choice(_NOUN)}-{random.randint(1, 99)}"


def generate_token() -> str:
    return secrets.token_hex(20)


def token_hash(token: str) -> str:
    return hashlib.sha256(token.encode()).hexdigest()


def generate_rsa_key_pair(comment: str = "dstack") -> Tuple[str, str]:
    """(private_pem, public_openssh) via ssh-keygen (no paramiko/cryptography in the image)."""
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "key")
        subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-C", comment, "-f", path], check=True,
                       capture_output=True)
        with open(path) as f:
            private = f.read()
        with open(path + ".pub") as f:
            public = f.read().strip()
    return private, public


def batched(items: List[T], n: int) -> Iterable[List[T]]:
    for i in range(0, len(items), n):
        yield items[i:i + n]


def get_or_error(v: Optional[T]) -> T:
    if v is None:
        raise ValueError("Optional value is None")
    return v


def pretty_resources(cpus=None, memory=None, gpu_count=None, gpu_name=None, gpu_memory=None, disk_size=None,
                     total_gpu_memory=None, compute_capability=None) -> str:
    parts = []
    if cpus is not None:
        parts.append(f"{cpus}xCPU")
    if memory is not None:
        parts.append(f"{memory}")
    if gpu_count:
        g = f"{gpu_count}x{gpu_name or 'GPU'}"
        if gpu_memory is not None:
            g += f" ({gpu_memory})"
        parts.append(g)
    if disk_size is not None:
        parts.append(f"{disk_size} (disk)")
    return ", ".join(parts)


def get_ip_from_network(network: Optional[str], addresses: List[str]) -> Optional[str]:
    """Pick the first host address (``ip/iface``) inside ``network`` (reference:
    ``utils/network.py``); without a network, the first private address."""
    ips = []
    for a in addresses:
        ip = a.split("/")[0].split("%")[0]  # drop the prefix length / IPv6 zone index
        try:
            ips.append(ipaddress.ip_address(ip))
        except ValueError:
            continue
    if network:
        net = ipaddress.ip_network(network, strict=False)
        for ip in ips:
            if ip.version == net.version and ip in net:
                return str(ip)
        return None
    for ip in ips:
        if ip.is_private:
            return str(ip)
    return str(ips[0]) if ips else None


def now_ts() -> float:
    return datetime.now(timezone.utc).timestamp()


def timedelta_seconds(td: timedelta) -> float:
    return td.total_seconds()
