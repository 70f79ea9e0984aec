"""Container images for AMD Instinct runs, and the ROCm floor of each accelerator generation.

The reference pins one base image to the accelerator stack it supports
(``/root/reference/docker/base/Dockerfile:1-30``, ``server/services/jobs/configurators/base.py:45-49``:
``dstackai/base:py<ver>-<tag>-cuda-12.1``).  Here the stack is ROCm + PyTorch-ROCm, and the
MI350-series (gfx950: MI350X, MI355X) needs ROCm 7.0 or newer -- a ROCm 6.x userspace has no gfx950
code objects in rocBLAS/hipBLASLt/MIOpen/RCCL and no gfx950 target in its compiler, so PyTorch
falls over at the first kernel.  ``DEFAULT_ROCM_IMAGE`` is the one image every MI355X default uses
(the job configurator, the container backends, ``docker/base/Dockerfile``, the examples).

The numbers in ``docs/performance.md`` were built and measured with ROCm 7.2 / PyTorch 2.10; this
repo's code needs ROCm >= 7.0 for gfx950 (``python -m dstack_amd.ops.build`` checks that hipcc
can target gfx950) and PyTorch >= 2.4 (``init_process_group(device_id=...)``).
"""

from __future__ import annotations

import re
from typing import Iterable, Optional, Tuple

DEFAULT_ROCM_IMAGE = "rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1"

# minimum ROCm (major, minor) per GPU name (case-insensitive); GPUs not listed have no floor here
MIN_ROCM = {
    "MI355X": (7, 0),
    "MI350X": (7, 0),
    "MI325X": (6, 2),
    "MI300X": (6, 0),
    "MI300A": (6, 0),
}

# ``rocm6.4_ubuntu...``, ``rocm-6.4.1``, ``rocm7.0.2``: the ROCm version a tag names
_TAG_ROCM = re.compile(r"rocm[-_]?(\d+)\.(\d+)", re.IGNORECASE)
# ``rocm/dev-ubuntu-22.04:6.4`` / ``rocm/rocm-terminal:7.0``: AMD's own ROCm repos put the version
# alone in the tag
_BARE_VERSION = re.compile(r"^(\d+)\.(\d+)(?:\.\d+)?(?:[-_].*)?$")


def image_rocm_version(image: Optional[str]) -> Optional[Tuple[int, int]]:
    """The ROCm version an image reference names in its tag, or None when the tag does not say
    (``latest``, a digest, a non-ROCm image): such images are never rejected here."""
    if not image:
        return None
    ref = image.split("@", 1)[0]
    name, _, tag = ref.rpartition(":")
    if not name or "/" in tag:  # no tag (the colon was a registry port)
        return None
    m = _TAG_ROCM.search(tag)
    if m:
        return int(m.group(1)), int(m.group(2))
    repo = name.rsplit("/", 1)[-1]
    if name.startswith("rocm/") and repo in ("dev-ubuntu-22.04", "dev-ubuntu-24.04", "dev-ubuntu-20.04",
                                             "rocm-terminal", "dev-centos-7", "dev-almalinux-8"):
        m = _BARE_VERSION.match(tag)
        if m:
            return int(m.group(1)), int(m.group(2))
    return None


def min_rocm_for(gpu_name: str) -> Optional[Tuple[int, int]]:
    return MIN_ROCM.get(gpu_name.upper())


def image_supports_gpu(image: Optional[str], gpu_name: str) -> bool:
    have = image_rocm_version(image)
    need = min_rocm_for(gpu_name)
    return have is None or need is None or have >= need


def unsupported_message(image: str, gpu_names: Iterable[str]) -> str:
    have = image_rocm_version(image)
    names = sorted({n.upper() for n in gpu_names})
    need = max(min_rocm_for(n) or (0, 0) for n in names)
    return (f"image {image} ships ROCm {have[0]}.{have[1]}, but {'/'.join(names)} (gfx950) needs ROCm "
            f">= {need[0]}.{need[1]}: use {DEFAULT_ROCM_IMAGE} or another ROCm >= {need[0]}.{need[1]} image")


def check_requested_gpus(image: Optional[str], gpu_names: Optional[Iterable[str]]) -> Optional[str]:
    """Configurator rule: when EVERY GPU name the run accepts needs a newer ROCm than the image's
    tag names, the run can never work -- the error message; otherwise None (runs that also accept
    older GPUs are placed only on those, see ``offer_supported``)."""
    names = [n for n in (gpu_names or []) if n]
    if not image or not names:
        return None
    if all(not image_supports_gpu(image, n) for n in names):
        return unsupported_message(image, names)
    return None


def offer_supported(image: Optional[str], gpus) -> bool:
    """Placement rule: an offer (or pool instance) whose GPUs need a newer ROCm than the job's
    image is skipped, so an unnamed ``gpu: 8`` request with a ROCm 6 image lands on MI300X-class
    hosts instead of failing at the first kernel on an MI355X."""
    return all(image_supports_gpu(image, g.name) for g in (gpus or []))
