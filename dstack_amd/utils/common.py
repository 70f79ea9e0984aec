"""Small shared helpers (reference: ``src/dstack/_internal/utils/common.py``,
``random_names.py``, ``crypto.py``, ``network.py``)."""

from __future__ import annotations

import hashlib
import ipaddress
import os
import random
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
    if dt is None:
        return "-"
    now = now or get_current_datetime()
    if dt.tzinfo is not None:
        dt = dt.astimezone(timezone.utc).replace(tzinfo=None)
    diff = now - dt
    s = int(diff.total_seconds())
    if s < 0:
        return "now"
    if s < 60:
        return f"{s} sec ago"
    if s < 3600:
        return f"{s // 60} min ago"
    if s < 86400:
        return f"{s // 3600} hour{'s' if s // 3600 > 1 else ''} ago"
    days = s // 86400
    if days < 7:
        return "yesterday" if days == 1 else f"{days} days ago"
    return dt.strftime("%b %d, %Y")


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
        ip = a.split("/")[0]
        try:
            ips.append(ipaddress.ip_address(ip))
        except ValueError:
            continue
    if network:
        net = ipaddress.ip_network(network, strict=False)
        for ip in ips:
            if ip in net:
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
