"""GPU knowledge base, AMD Instinct first.

Replaces the reference's dependence on ``gpuhunt`` for GPU facts and the name normalisers of
``src/dstack/_internal/utils/gpu.py:4-59`` (nvidia-smi / amd-smi ``market_name`` / hl-smi → catalog
names). Adds what the MI355X scheduler needs: HBM size and bandwidth, dense MFMA peaks, the xGMI
link count and the gfx target per model.
"""

from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Dict, Optional

from dstack_amd.core.models.resources import AcceleratorVendor


@dataclass(frozen=True)
class GPUInfo:
    name: str
    vendor: AcceleratorVendor
    memory_gb: float
    hbm_tb_s: float = 0.0
    bf16_dense_tflops: float = 0.0
    fp8_dense_tflops: float = 0.0
    xgmi_links: int = 0  # peer links per GPU (AMD Infinity Fabric / xGMI)
    xgmi_link_gb_s: float = 0.0  # per direction
    arch: str = ""
    compute_capability: Optional[tuple] = None


_AMD = AcceleratorVendor.AMD
_NV = AcceleratorVendor.NVIDIA

GPUS: Dict[str, GPUInfo] = {
    g.name: g
    for g in [
        # AMD Instinct (CDNA)
        GPUInfo("MI355X", _AMD, 288, 8.0, 2500, 5000, 7, 153.6, "gfx950"),
        GPUInfo("MI350X", _AMD, 288, 8.0, 2300, 4600, 7, 153.6, "gfx950"),
        GPUInfo("MI325X", _AMD, 256, 6.0, 1307, 2615, 7, 128.0, "gfx942"),
        GPUInfo("MI300X", _AMD, 192, 5.3, 1307, 2615, 7, 128.0, "gfx942"),
        GPUInfo("MI300A", _AMD, 128, 5.3, 981, 1961, 7, 128.0, "gfx942"),
        GPUInfo("MI250X", _AMD, 128, 3.2, 383, 0, 8, 50.0, "gfx90a"),
        GPUInfo("MI250", _AMD, 128, 3.2, 362, 0, 6, 50.0, "gfx90a"),
        GPUInfo("MI210", _AMD, 64, 1.6, 181, 0, 3, 50.0, "gfx90a"),
        GPUInfo("MI100", _AMD, 32, 1.2, 92, 0, 3, 46.0, "gfx908"),
        # NVIDIA (so that non-AMD offers are still describable)
        GPUInfo("H200", _NV, 141, 4.8, 989, 1979, 18, 50.0, "sm90", (9, 0)),
        GPUInfo("H100", _NV, 80, 3.35, 989, 1979, 18, 50.0, "sm90", (9, 0)),
        GPUInfo("A100", _NV, 80, 2.0, 312, 0, 12, 50.0, "sm80", (8, 0)),
        GPUInfo("L40S", _NV, 48, 0.86, 362, 733, 0, 0, "sm89", (8, 9)),
        GPUInfo("A10G", _NV, 24, 0.6, 70, 0, 0, 0, "sm86", (8, 6)),
        GPUInfo("L4", _NV, 24, 0.3, 121, 242, 0, 0, "sm89", (8, 9)),
        GPUInfo("T4", _NV, 16, 0.3, 65, 0, 0, 0, "sm75", (7, 5)),
    ]
}


def gpu_info(name: str) -> Optional[GPUInfo]:
    return GPUS.get(name) or GPUS.get(name.upper())


# NVIDIA model names without catalog facts: enough to tell the vendor of a ``resources.gpu`` name
_NVIDIA_NAMES = frozenset(n.upper() for n in (
    "B200", "GB200", "H200", "H100", "H100NVL", "H800", "GH200", "A100", "A800", "A40", "A30", "A10", "A10G",
    "A16", "A2", "A4000", "A4500", "A5000", "A6000", "A1000", "A2000", "RTX6000", "RTX4000", "RTX5000",
    "RTXA6000", "RTXA5000", "RTXA4000", "L40", "L40S", "L4", "L20", "T4", "V100", "P100", "P40", "P4", "K80",
    "RTX3090", "RTX4090", "RTX3080", "RTX4080"))


def vendor_of(name: str) -> Optional[AcceleratorVendor]:
    info = gpu_info(name)
    if info:
        return info.vendor
    if name.upper().replace("-", "") in _NVIDIA_NAMES:
        return _NV
    if re.match(r"^MI\d", name, re.I):
        return _AMD
    if re.match(r"^(v\d|tpu)", name, re.I):
        return AcceleratorVendor.GOOGLE
    if name.lower().startswith("gaudi"):
        return AcceleratorVendor.INTEL
    return None


_AMD_MARKET_NAME = re.compile(
    r"^(?:AMD )?(?:Instinct )?(?P<name>MI\d{1,3}[A-Z]?(?:-\w+)?)(?:\s|$)", flags=re.ASCII | re.I
)

# amd-smi reports e.g. "AMD Instinct MI355 OAM" for the MI355X
_AMD_ALIASES = {"MI300X-O": "MI300X", "MI355": "MI355X", "MI350": "MI350X", "MI325": "MI325X"}


def convert_amd_gpu_name(name: str) -> str:
    """amd-smi ``asic.market_name`` → catalog name (``AMD Instinct MI355 OAM`` → ``MI355X``)."""
    m = _AMD_MARKET_NAME.search(name.strip())
    if m:
        name = m.group("name").upper()
    return _AMD_ALIASES.get(name, name)


def convert_nvidia_gpu_name(name: str) -> str:
    name = name.replace("NVIDIA ", "").replace("Tesla ", "").replace("Quadro ", "").replace("GeForce ", "")
    if "GH200" in name:
        return "GH200"
    if "RTX A" in name:
        m = re.search(r"(A\d+)", name.replace("RTX A", "A"))
        return m.group(0) if m else name.replace(" ", "")
    name = name.replace(" Ti", "Ti").replace(" NVL", "NVL").replace(" Ada Generation", "Ada").replace("RTX ", "RTX")
    m = re.search(r"([AHLPTV]\d+\w*)", name)
    return m.group(0) if m else name.replace(" ", "")


_INTEL_GAUDI = {"HL-205": "Gaudi", "HL-225": "Gaudi2", "HL-325": "Gaudi3", "HL-338": "Gaudi3"}


def convert_intel_accelerator_name(name: str) -> str:
    for model, market in _INTEL_GAUDI.items():
        if name.startswith(model):
            return market
    return name


def normalize_gpu_name(name: str) -> str:
    """Any vendor's marketing/device-plugin name → catalog name (AMD first)."""
    if not name:
        return name
    up = name.upper()
    if "AMD" in up or "INSTINCT" in up or re.match(r"^MI\d", up):
        return convert_amd_gpu_name(name)
    if up.startswith("HL-"):
        return convert_intel_accelerator_name(name)
    return convert_nvidia_gpu_name(name)
