"""Offline offer catalog for cloud backends (replaces ``gpuhunt``; reference:
``C/backends/base/offers.py:18-175``).

The MI355X build is AMD-first: the catalog lists the clouds' Instinct instance types (MI300X,
MI325X, MI355X) next to a few NVIDIA/CPU types.  Prices are list prices (USD/h, on-demand) used
for ordering offers; they are informational only.  Provisioning against a cloud API requires the
backend's credentials and network access; in an air-gapped deployment cloud backends still plan
(offers) but ``run_job`` raises ``BackendNotAvailable``.
"""

from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Dict, List, Optional

from dstack_amd.core.backends.base import Compute, offer_matches
from dstack_amd.core.errors import BackendNotAvailable
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.gpus import gpu_info
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


@dataclass(frozen=True)
class CatalogItem:
    backend: BackendType
    instance_name: str
    regions: tuple
    cpus: int
    memory_gb: int
    gpu_name: Optional[str]
    gpu_count: int
    price: float
    spot_price: Optional[float] = None
    disk_gb: int = 100


_B = BackendType
CATALOG: List[CatalogItem] = [
    # AMD Instinct
    CatalogItem(_B.VULTR, "vbm-256c-2048gb-8-mi355x-gpu", ("ewr", "atl"), 256, 3072, "MI355X", 8, 21.60, disk_gb=15000),
    CatalogItem(_B.VULTR, "vbm-256c-2048gb-8-mi325x-gpu", ("ewr",), 256, 2048, "MI325X", 8, 17.52, disk_gb=15000),
    CatalogItem(_B.VULTR, "vbm-256c-2048gb-8-mi300x-gpu", ("ewr", "ord"), 256, 2048, "MI300X", 8, 15.92, disk_gb=15000),
    CatalogItem(_B.OCI, "BM.GPU.MI300X.8", ("us-chicago-1",), 112, 2048, "MI300X", 8, 48.0, disk_gb=30000),
    CatalogItem(_B.OCI, "BM.GPU.MI355X.8", ("us-chicago-1",), 128, 3072, "MI355X", 8, 60.0, disk_gb=30000),
    CatalogItem(_B.AZURE, "Standard_ND96isr_MI300X_v5", ("eastus", "westus"), 96, 1850, "MI300X", 8, 48.0,
                disk_gb=1000),
    CatalogItem(_B.RUNPOD, "1x-MI300X", ("EU-RO-1", "US-TX-3"), 24, 283, "MI300X", 1, 2.49, 1.99),
    CatalogItem(_B.RUNPOD, "8x-MI300X", ("EU-RO-1",), 192, 2264, "MI300X", 8, 19.92),
    CatalogItem(_B.TENSORDOCK, "mi300x-8", ("us",), 192, 1536, "MI300X", 8, 18.0),
    CatalogItem(_B.CUDO, "epyc-genoa-mi300x", ("no-luster-1",), 96, 1024, "MI300X", 4, 10.0),
    # NVIDIA / CPU reference types
    CatalogItem(_B.AWS, "p5.48xlarge", ("us-east-1", "us-west-2"), 192, 2048, "H100", 8, 98.32, 39.33, 3000),
    CatalogItem(_B.AWS, "g5.xlarge", ("us-east-1", "eu-west-1"), 4, 16, "A10G", 1, 1.006, 0.39),
    CatalogItem(_B.AWS, "c6i.xlarge", ("us-east-1",), 4, 8, None, 0, 0.17, 0.07),
    CatalogItem(_B.GCP, "a3-highgpu-8g", ("us-central1",), 208, 1872, "H100", 8, 88.49, 35.0, 3000),
    CatalogItem(_B.GCP, "e2-standard-4", ("us-central1",), 4, 16, None, 0, 0.134, 0.04),
    CatalogItem(_B.LAMBDA, "gpu_8x_h100_sxm5", ("us-east-1",), 208, 1800, "H100", 8, 23.92),
    CatalogItem(_B.DATACRUNCH, "8H100.80S.176V", ("FIN-01",), 176, 1480, "H100", 8, 21.92),
    CatalogItem(_B.NEBIUS, "gpu-h100-sxm-8", ("eu-north1",), 128, 1600, "H100", 8, 23.6),
    CatalogItem(_B.VASTAI, "vast-1xA100", ("any",), 16, 64, "A100", 1, 1.1),
    CatalogItem(_B.KUBERNETES, "k8s-node", ("-",), 8, 32, None, 0, 0.0),
    CatalogItem(_B.DSTACK, "dstack-mi300x", ("any",), 24, 283, "MI300X", 1, 2.49),
]


def catalog_offers(backend: BackendType, regions: Optional[List[str]] = None,
                   requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
    out = []
    for it in CATALOG:
        if it.backend != backend:
            continue
        info = gpu_info(it.gpu_name) if it.gpu_name else None
        gpus = [Gpu(name=it.gpu_name, memory_mib=int((info.memory_gb if info else 0) * 1024),
                    vendor=info.vendor if info else None) for _ in range(it.gpu_count)] if it.gpu_name else []
        for spot in ([False, True] if it.spot_price is not None else [False]):
            for region in it.regions:
                if regions and region not in regions:
                    continue
                res = Resources(cpus=it.cpus, memory_mib=it.memory_gb * 1024, gpus=gpus, spot=spot,
                                disk=Disk(size_mib=it.disk_gb * 1024))
                offer = InstanceOfferWithAvailability(
                    backend=backend, instance=InstanceType(name=it.instance_name, resources=res), region=region,
                    price=it.spot_price if spot else it.price, availability=InstanceAvailability.UNKNOWN,
                )
                if offer_matches(offer, requirements):
                    out.append(offer)
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
