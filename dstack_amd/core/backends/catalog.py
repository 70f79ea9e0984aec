"""Offer catalog for cloud backends (replaces ``gpuhunt``; reference:
``C/backends/base/offers.py:18-175``).

Three layers, queried per backend, each falling back to the next:

1. **online** -- the backend's own live listing (``Compute._fetch_catalog``: Lambda
   ``/instance-types``, Vultr plans + region availability, DataCrunch instance types +
   availability, TensorDock host nodes, RunPod GPU types per data centre, AWS instance-type
   offerings + current spot prices, Azure retail prices).  Rows carry the live price and an
   availability.  Results are cached in memory and on disk (``DSTACK_CATALOG_CACHE_DIR``) for
   ``DSTACK_CATALOG_ONLINE_TTL`` seconds; a failed refresh serves the last good listing for up to
   ``DSTACK_CATALOG_MAX_STALE`` seconds before dropping to the offline layer.
2. **offline** -- a downloaded catalog (``DSTACK_CATALOG_URL``: a zip of ``<provider>.csv``, or
   ``DSTACK_CATALOG_PATH``: a directory / zip on disk), refreshed once per
   ``DSTACK_CATALOG_OFFLINE_TTL``.  Same CSV columns as gpuhunt's catalog (``instance_name,
   location,price,cpu,memory,gpu_count,gpu_name,gpu_memory,spot,disk_size,gpu_vendor``).
3. **built-in** -- the table below (the clouds' Instinct MI300X / MI325X / MI355X types first, plus
   a few NVIDIA / CPU types), list prices in USD/h.

Disk size follows the reference's ``choose_disk_size_mib``: a row with a fixed disk keeps it (and
must fit the requested range); a row without one gets the requested minimum, clamped to the
backend's configurable range (no offer if the ranges do not intersect).
"""

from __future__ import annotations

import csv
import hashlib
import io
import json
import logging
import os
import threading
import time
import zipfile
from dataclasses import asdict, dataclass, replace
from pathlib import Path
from typing import Callable, Dict, Iterable, List, Optional, Tuple

from dstack_amd.core.backends.base import Compute, offer_matches
from dstack_amd.core.errors import BackendNotAvailable
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.gpus import gpu_info, normalize_gpu_name, vendor_of
from dstack_amd.core.models.instances import (
    Disk,
    Gpu,
    InstanceAvailability,
    InstanceConfiguration,
    InstanceOfferWithAvailability,
    InstanceType,
    Resources,
)
from dstack_amd.core.models.runs import JobProvisioningData, Requirements

logger = logging.getLogger(__name__)


@dataclass(frozen=True)
class CatalogItem:
    """One built-in instance type (expanded to a row per region and spot mode)."""

    backend: BackendType
    instance_name: str
    regions: tuple
    cpus: int
    memory_gb: int
    gpu_name: Optional[str]
    gpu_count: int
    price: float
    spot_price: Optional[float] = None
    disk_gb: Optional[int] = None  # fixed local disk (bare metal); None: configurable at launch


@dataclass(frozen=True)
class CatalogRow:
    """One purchasable (instance type, location, spot) combination -- gpuhunt's ``CatalogItem``."""

    instance_name: str
    location: str
    price: float
    cpu: int
    memory_gb: float
    gpu_count: int = 0
    gpu_name: Optional[str] = None
    gpu_memory_gb: Optional[float] = None
    spot: bool = False
    disk_gb: Optional[float] = None  # None: the disk is configurable at launch
    gpu_vendor: Optional[str] = None
    availability: InstanceAvailability = InstanceAvailability.UNKNOWN

    def to_json(self) -> dict:
        d = asdict(self)
        d["availability"] = self.availability.value
        return d

    @classmethod
    def from_json(cls, d: dict) -> "CatalogRow":
        d = dict(d)
        d["availability"] = InstanceAvailability(d.get("availability", "unknown"))
        return cls(**d)


def gpu_row(instance_name: str, location: str, price: float, cpu: int, memory_gb: float, gpu_name: Optional[str],
            gpu_count: int, *, spot: bool = False, disk_gb: Optional[float] = None,
            gpu_memory_gb: Optional[float] = None,
            availability: InstanceAvailability = InstanceAvailability.UNKNOWN) -> CatalogRow:
    """Row with the GPU name normalised and its memory / vendor filled from the GPU table."""
    name = normalize_gpu_name(gpu_name) if gpu_name else None
    info = gpu_info(name) if name else None
    vendor = info.vendor if info else (vendor_of(name) if name else None)
    return CatalogRow(
        instance_name=instance_name, location=location, price=round(float(price), 6), cpu=int(cpu),
        memory_gb=float(memory_gb), gpu_count=int(gpu_count) if name else 0, gpu_name=name if gpu_count else None,
        gpu_memory_gb=gpu_memory_gb if gpu_memory_gb is not None else (info.memory_gb if info else None),
        spot=spot, disk_gb=disk_gb, gpu_vendor=vendor.value if vendor is not None else None,
        availability=availability,
    )


_B = BackendType
CATALOG: List[CatalogItem] = [
    # AMD Instinct
    CatalogItem(_B.VULTR, "vbm-256c-2048gb-8-mi355x-gpu", ("ewr", "atl"), 256, 3072, "MI355X", 8, 21.60, disk_gb=15000),
    CatalogItem(_B.VULTR, "vbm-256c-2048gb-8-mi325x-gpu", ("ewr",), 256, 2048, "MI325X", 8, 17.52, disk_gb=15000),
    CatalogItem(_B.VULTR, "vbm-256c-2048gb-8-mi300x-gpu", ("ewr", "ord"), 256, 2048, "MI300X", 8, 15.92, disk_gb=15000),
    CatalogItem(_B.OCI, "BM.GPU.MI300X.8", ("us-chicago-1",), 112, 2048, "MI300X", 8, 48.0),
    CatalogItem(_B.OCI, "BM.GPU.MI355X.8", ("us-chicago-1",), 128, 3072, "MI355X", 8, 60.0),
    CatalogItem(_B.AZURE, "Standard_ND96isr_MI300X_v5", ("eastus", "westus"), 96, 1850, "MI300X", 8, 48.0),
    CatalogItem(_B.RUNPOD, "1x-MI300X", ("EU-RO-1", "US-TX-3"), 24, 283, "MI300X", 1, 2.49, 1.99),
    CatalogItem(_B.RUNPOD, "8x-MI300X", ("EU-RO-1",), 192, 2264, "MI300X", 8, 19.92),
    CatalogItem(_B.TENSORDOCK, "mi300x-8", ("us",), 192, 1536, "MI300X", 8, 18.0),
    CatalogItem(_B.CUDO, "epyc-genoa-mi300x", ("no-luster-1",), 96, 1024, "MI300X", 4, 10.0),
    # NVIDIA / CPU reference types
    CatalogItem(_B.AWS, "p5.48xlarge", ("us-east-1", "us-west-2"), 192, 2048, "H100", 8, 98.32, 39.33),
    CatalogItem(_B.AWS, "g5.xlarge", ("us-east-1", "eu-west-1"), 4, 16, "A10G", 1, 1.006, 0.39),
    CatalogItem(_B.AWS, "c6i.xlarge", ("us-east-1",), 4, 8, None, 0, 0.17, 0.07),
    CatalogItem(_B.GCP, "a3-highgpu-8g", ("us-central1",), 208, 1872, "H100", 8, 88.49, 35.0),
    CatalogItem(_B.GCP, "e2-standard-4", ("us-central1",), 4, 16, None, 0, 0.134, 0.04),
    CatalogItem(_B.LAMBDA, "gpu_8x_h100_sxm5", ("us-east-1",), 208, 1800, "H100", 8, 23.92),
    CatalogItem(_B.DATACRUNCH, "8H100.80S.176V", ("FIN-01",), 176, 1480, "H100", 8, 21.92),
    CatalogItem(_B.NEBIUS, "gpu-h100-sxm-8", ("eu-north1",), 128, 1600, "H100", 8, 23.6),
    CatalogItem(_B.VASTAI, "vast-1xA100", ("any",), 16, 64, "A100", 1, 1.1),
    CatalogItem(_B.KUBERNETES, "k8s-node", ("-",), 8, 32, None, 0, 0.0),
    CatalogItem(_B.DSTACK, "dstack-mi300x", ("any",), 24, 283, "MI300X", 1, 2.49),
]


def builtin_rows(backend: BackendType) -> List[CatalogRow]:
    out = []
    for it in CATALOG:
        if it.backend != backend:
            continue
        for spot in ([False, True] if it.spot_price is not None else [False]):
            for region in it.regions:
                out.append(gpu_row(it.instance_name, region, it.spot_price if spot else it.price, it.cpus,
                                   it.memory_gb, it.gpu_name, it.gpu_count, spot=spot, disk_gb=it.disk_gb))
    return out


# ---------------------------------------------------------------------------------------------
# offline catalog (downloaded CSV zip)
# ---------------------------------------------------------------------------------------------
CSV_COLUMNS = ("instance_name", "location", "price", "cpu", "memory", "gpu_count", "gpu_name", "gpu_memory", "spot",
               "disk_size", "gpu_vendor")


def provider_name(backend: BackendType) -> str:
    """File / provider name of a backend in the catalog (gpuhunt calls Lambda ``lambdalabs``)."""
    return "lambdalabs" if backend == BackendType.LAMBDA else backend.value


def _f(v: str) -> Optional[float]:
    v = (v or "").strip()
    return float(v) if v else None


def parse_catalog_csv(text: str) -> List[CatalogRow]:
    rows = []
    for rec in csv.DictReader(io.StringIO(text)):
        try:
            gpu_count = int(_f(rec.get("gpu_count", "")) or 0)
            rows.append(gpu_row(
                rec["instance_name"], rec["location"], float(rec["price"]), int(_f(rec.get("cpu", "")) or 0),
                _f(rec.get("memory", "")) or 0.0, rec.get("gpu_name") or None, gpu_count,
                spot=(rec.get("spot", "").strip().lower() in ("true", "1", "yes")),
                disk_gb=_f(rec.get("disk_size", "")), gpu_memory_gb=_f(rec.get("gpu_memory", "")),
            ))
        except (KeyError, ValueError) as e:
            logger.debug("catalog: skipping malformed row %s: %s", rec, e)
    return rows


def dump_catalog_csv(rows: Iterable[CatalogRow]) -> str:
    buf = io.StringIO()
    w = csv.writer(buf)
    w.writerow(CSV_COLUMNS)
    for r in rows:
        w.writerow([r.instance_name, r.location, r.price, r.cpu, r.memory_gb, r.gpu_count, r.gpu_name or "",
                    "" if r.gpu_memory_gb is None else r.gpu_memory_gb, str(r.spot).lower(),
                    "" if r.disk_gb is None else r.disk_gb, r.gpu_vendor or ""])
    return buf.getvalue()


def cache_dir() -> Path:
    return Path(os.getenv("DSTACK_CATALOG_CACHE_DIR", str(Path.home() / ".dstack" / "catalog")))


class OfflineCatalog:
    """Per-provider rows from a catalog zip / directory, downloaded at most once per TTL."""

    def __init__(self, url: Optional[str] = None, path: Optional[str] = None, ttl: Optional[float] = None,
                 fetch: Optional[Callable[[str], bytes]] = None):
        self.url = url if url is not None else os.getenv("DSTACK_CATALOG_URL")
        self.path = path if path is not None else os.getenv("DSTACK_CATALOG_PATH")
        self.ttl = ttl if ttl is not None else float(os.getenv("DSTACK_CATALOG_OFFLINE_TTL", 24 * 3600))
        self._fetch = fetch or _http_get_bytes
        self._lock = threading.Lock()
        self._loaded_at = 0.0
        self._files: Dict[str, str] = {}

    def configured(self) -> bool:
        return bool(self.url or self.path)

    def rows(self, backend: BackendType) -> Optional[List[CatalogRow]]:
        if not self.configured():
            return None
        with self._lock:
            if not self._files or time.time() - self._loaded_at > self.ttl:
                self._reload()
            text = self._files.get(provider_name(backend))
        return parse_catalog_csv(text) if text is not None else None

    def _reload(self) -> None:
        try:
            if self.path:
                self._files = _read_catalog_source(Path(self.path))
            else:
                self._files = self._download()
            self._loaded_at = time.time()
        except Exception as e:  # noqa: BLE001 -- keep the previous catalog, retry after a minute
            logger.warning("catalog: cannot load offline catalog: %s", e)
            self._loaded_at = time.time() - self.ttl + 60

    def _download(self) -> Dict[str, str]:
        dest = cache_dir() / ("offline-" + hashlib.sha256(self.url.encode()).hexdigest()[:16] + ".zip")
        if dest.exists() and time.time() - dest.stat().st_mtime < self.ttl:
            return _read_catalog_source(dest)
        try:
            data = self._fetch(self.url)
            _read_zip(data)  # validate before replacing the cached copy
            dest.parent.mkdir(parents=True, exist_ok=True)
            tmp = dest.with_suffix(".tmp")
            tmp.write_bytes(data)
            os.replace(tmp, dest)
        except Exception:
            if dest.exists():  # stale but good
                logger.warning("catalog: download of %s failed, using the cached copy", self.url)
                return _read_catalog_source(dest)
            raise
        return _read_catalog_source(dest)


def _read_zip(data: bytes) -> Dict[str, str]:
    with zipfile.ZipFile(io.BytesIO(data)) as z:
        return {Path(n).stem: z.read(n).decode() for n in z.namelist() if n.endswith(".csv")}


def _read_catalog_source(p: Path) -> Dict[str, str]:
    if p.is_dir():
        return {f.stem: f.read_text() for f in sorted(p.glob("*.csv"))}
    return _read_zip(p.read_bytes())


def _http_get_bytes(url: str) -> bytes:
    import httpx

    r = httpx.get(url, timeout=60, follow_redirects=True)
    r.raise_for_status()
    return r.content


# ---------------------------------------------------------------------------------------------
# online listings (per backend credentials), memory + disk cache with stale fallback
# ---------------------------------------------------------------------------------------------
class OnlineCache:
    def __init__(self, ttl: Optional[float] = None, max_stale: Optional[float] = None, directory: Optional[Path] = None):
        self.ttl = ttl if ttl is not None else float(os.getenv("DSTACK_CATALOG_ONLINE_TTL", 300))
        self.max_stale = max_stale if max_stale is not None else float(os.getenv("DSTACK_CATALOG_MAX_STALE", 86400))
        self.directory = directory
        # after a failed live fetch the key is not fetched again for this long (serving cached or
        # offline rows meanwhile): an unreachable API must not stall every plan / scheduler pass
        self.failure_backoff = min(self.ttl, float(os.getenv("DSTACK_CATALOG_FAILURE_BACKOFF", 60)))
        self._failed: Dict[str, float] = {}
        self._mem: Dict[str, Tuple[float, List[CatalogRow]]] = {}
        self._locks: Dict[str, threading.Lock] = {}
        self._guard = threading.Lock()

    def _dir(self) -> Path:
        return self.directory or cache_dir()

    def _path(self, key: str) -> Path:
        return self._dir() / f"online-{hashlib.sha256(key.encode()).hexdigest()[:24]}.json"

    def _load_disk(self, key: str) -> Optional[Tuple[float, List[CatalogRow]]]:
        try:
            d = json.loads(self._path(key).read_text())
            return float(d["fetched_at"]), [CatalogRow.from_json(r) for r in d["rows"]]
        except (OSError, ValueError, KeyError, TypeError):
            return None

    def _store(self, key: str, at: float, rows: List[CatalogRow]) -> None:
        self._mem[key] = (at, rows)
        try:
            p = self._path(key)
            p.parent.mkdir(parents=True, exist_ok=True)
            tmp = p.with_suffix(".tmp")
            tmp.write_text(json.dumps({"key_hash": p.stem, "fetched_at": at, "rows": [r.to_json() for r in rows]}))
            os.replace(tmp, p)
        except OSError as e:
            logger.debug("catalog: cannot persist %s: %s", key, e)

    def get(self, key: str, fetch: Callable[[], List[CatalogRow]]) -> Optional[List[CatalogRow]]:
        """Fresh cached rows, else a refresh; on refresh failure the last good rows within
        ``max_stale``; ``None`` when there is nothing usable."""
        with self._guard:
            lock = self._locks.setdefault(key, threading.Lock())
        with lock:  # one refresh per key at a time
            hit = self._mem.get(key) or self._load_disk(key)
            now = time.time()
            if hit and now - hit[0] < self.ttl:
                self._mem[key] = hit
                return hit[1]
            failed_at = self._failed.get(key)
            if failed_at is not None and now - failed_at < self.failure_backoff:
                return hit[1] if hit and now - hit[0] < self.max_stale else None  # negative cache
            try:
                rows = fetch()
            except Exception as e:  # noqa: BLE001 -- any API failure degrades to cached/offline data
                self._failed[key] = now
                if hit and now - hit[0] < self.max_stale:
                    logger.warning("catalog: live listing %s failed (%s); serving data %.0fs old", key, e, now - hit[0])
                    return hit[1]
                logger.warning("catalog: live listing %s failed (%s); using the offline catalog for %.0fs", key, e,
                               self.failure_backoff)
                return None
            self._failed.pop(key, None)
            self._store(key, now, rows)
            return rows


_offline = OfflineCatalog()
_online = OnlineCache()


def catalog_fetch_timeout() -> float:
    """Per-request HTTP timeout (s) of live catalog listings (``DSTACK_CATALOG_FETCH_TIMEOUT``,
    default 10): a listing feeds a plan, so it must fail fast, unlike a launch call."""
    return float(os.getenv("DSTACK_CATALOG_FETCH_TIMEOUT", 10))


def reset_catalog_state() -> None:
    """Re-read the environment (tests, or after changing ``DSTACK_CATALOG_*``)."""
    global _offline, _online
    _offline = OfflineCatalog()
    _online = OnlineCache()


def offline_rows(backend: BackendType) -> List[CatalogRow]:
    rows = _offline.rows(backend)
    return rows if rows is not None else builtin_rows(backend)


def catalog_rows(backend: BackendType, fetch: Optional[Callable[[], List[CatalogRow]]] = None,
                 cache_key: Optional[str] = None) -> Tuple[List[CatalogRow], str]:
    """Rows for one backend and the layer they came from (``online`` / ``offline``)."""
    if fetch is not None:
        rows = _online.get(cache_key or provider_name(backend), fetch)
        if rows is not None:
            return rows, "online"
    return offline_rows(backend), "offline"


# ---------------------------------------------------------------------------------------------
# rows -> offers
# ---------------------------------------------------------------------------------------------
def choose_disk_size_gb(row_disk_gb: Optional[float], requirements: Optional[Requirements],
                        configurable: Tuple[float, Optional[float]] = (1.0, None), default_gb: float = 100.0
                        ) -> Optional[float]:
    """Reference ``choose_disk_size_mib``: fixed disks must fit the request; configurable disks take
    the requested minimum clamped to the backend's range (``None``: no intersection)."""
    req = requirements.resources.disk.size if requirements and requirements.resources.disk else None
    if row_disk_gb:
        if req is not None and not req.contains(row_disk_gb):
            return None
        return float(row_disk_gb)
    lo = req.min if req is not None and req.min is not None else default_gb
    hi = req.max if req is not None else None
    lo = max(lo, configurable[0])
    if configurable[1] is not None:
        hi = configurable[1] if hi is None else min(hi, configurable[1])
    if hi is not None and lo > hi:
        return None
    return float(lo)


def row_to_offer(backend: BackendType, row: CatalogRow, requirements: Optional[Requirements] = None,
                 configurable_disk: Tuple[float, Optional[float]] = (1.0, None)
                 ) -> Optional[InstanceOfferWithAvailability]:
    disk_gb = choose_disk_size_gb(row.disk_gb, requirements, configurable_disk)
    if disk_gb is None:
        return None
    gpus = []
    if row.gpu_count and row.gpu_name:
        gpus = [Gpu(name=row.gpu_name, memory_mib=int(round((row.gpu_memory_gb or 0) * 1024)),
                    vendor=row.gpu_vendor)] * row.gpu_count
    res = Resources(cpus=row.cpu, memory_mib=int(round(row.memory_gb * 1024)), gpus=gpus, spot=row.spot,
                    disk=Disk(size_mib=int(round(disk_gb * 1024))))
    return InstanceOfferWithAvailability(
        backend=backend, instance=InstanceType(name=row.instance_name, resources=res), region=row.location,
        price=row.price, availability=row.availability,
    )


def get_catalog_offers(backend: BackendType, locations: Optional[List[str]] = None,
                       requirements: Optional[Requirements] = None,
                       configurable_disk: Tuple[float, Optional[float]] = (1.0, None),
                       extra_filter: Optional[Callable[[InstanceOfferWithAvailability], bool]] = None,
                       fetch: Optional[Callable[[], List[CatalogRow]]] = None, cache_key: Optional[str] = None,
                       rows: Optional[List[CatalogRow]] = None) -> List[InstanceOfferWithAvailability]:
    """Offers of one backend that match ``requirements`` (reference ``get_catalog_offers``)."""
    if rows is None:
        rows, _ = catalog_rows(backend, fetch, cache_key)
    out = []
    for row in rows:
        if locations and row.location not in locations:
            continue
        offer = row_to_offer(backend, row, requirements, configurable_disk)
        if offer is None or not offer_matches(offer, requirements):
            continue
        if extra_filter is not None and not extra_filter(offer):
            continue
        out.append(offer)
    return out


def catalog_offers(backend: BackendType, regions: Optional[List[str]] = None,
                   requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
    """Offline-layer offers (downloaded catalog, else the built-in table)."""
    return get_catalog_offers(backend, regions, requirements)


def merge_live(rows: List[CatalogRow], live: Dict[Tuple[str, str, bool], Tuple[Optional[float], InstanceAvailability]]
               ) -> List[CatalogRow]:
    """Overlay live ``(instance, location, spot) -> (price | None, availability)`` on rows."""
    out = []
    for r in rows:
        hit = live.get((r.instance_name, r.location, r.spot))
        if hit is None:
            out.append(r)
            continue
        price, avail = hit
        out.append(replace(r, price=price if price is not None else r.price, availability=avail))
    return out


class CatalogCompute(Compute):
    """Cloud backend that plans from the catalog; provisioning needs the cloud API."""

    def __init__(self, backend_type: BackendType, config: Dict, auth: Dict):
        super().__init__()
        self.TYPE = backend_type
        self.config = config
        self.auth = auth

    def get_offers(self, requirements: Optional[Requirements] = None):
        return catalog_offers(self.TYPE, self.config.get("regions"), requirements)

    def create_instance(self, instance_offer: InstanceOfferWithAvailability,
                        instance_config: InstanceConfiguration) -> JobProvisioningData:
        raise BackendNotAvailable(
            f"{self.TYPE.value}: provisioning requires the cloud API, which is unreachable from this server"
        )

    def terminate_instance(self, instance_id: str, region: str, backend_data: Optional[str] = None) -> None:
        return None

    def describe(self) -> str:
        return json.dumps({"type": self.TYPE.value, **self.config})
