"""One gfx950-capable image story (reference: ``docker/base/Dockerfile:1-30``,
``server/services/jobs/configurators/base.py:45-49``): every MI355X default and example uses a
ROCm >= 7.0 PyTorch image, the configurator rejects a run that only accepts MI350X/MI355X with an
image whose tag names ROCm 6.x, and placement skips gfx950 offers for such images."""

import glob
import os
import re

import pytest
import yaml

from dstack_amd.core.errors import ServerClientError
from dstack_amd.core.models import images
from dstack_amd.core.models.instances import Gpu
from dstack_amd.core.models.runs import RunSpec
from dstack_amd.server.services.jobs.configurators import DEFAULT_AMD_IMAGE, get_job_specs_from_run_spec

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("image,want", [
    ("rocm/pytorch:rocm6.4_ubuntu22.04_py3.10_pytorch_release_2.6.0", (6, 4)),
    ("rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1", (7, 0)),
    ("rocm/vllm:rocm6.3.1_vllm_0.8.5_20250513", (6, 3)),
    ("ghcr.io/huggingface/text-generation-inference:3.0.1-rocm", None),
    ("rocm/dev-ubuntu-22.04:6.4", (6, 4)),
    ("rocm/dev-ubuntu-22.04:7.0.2-complete", (7, 0)),
    ("rocm/pytorch:latest", None),
    ("rocm/pytorch", None),
    ("registry.local:5000/team/train", None),
    ("registry.local:5000/team/train:rocm-6.2", (6, 2)),
    ("python:3.10-slim", None),
    ("rocm/pytorch@sha256:abcd", None),
])
def test_image_rocm_version(image, want):
    assert images.image_rocm_version(image) == want


def test_default_image_is_gfx950_capable_everywhere():
    assert images.image_rocm_version(images.DEFAULT_ROCM_IMAGE) >= (7, 0)
    assert DEFAULT_AMD_IMAGE == images.DEFAULT_ROCM_IMAGE
    from dstack_amd.core.backends.clouds import containers

    assert containers.DEFAULT_ROCM_IMAGE == images.DEFAULT_ROCM_IMAGE
    with open(os.path.join(REPO, "docker", "base", "Dockerfile")) as f:
        m = re.search(r"ARG ROCM_IMAGE=(\S+)", f.read())
    assert m and m.group(1) == images.DEFAULT_ROCM_IMAGE


def _mi35x(conf) -> bool:
    res = conf.get("resources") or {}
    gpu = res.get("gpu")
    return isinstance(gpu, (str, dict)) and re.search(r"MI35[05]X", str(gpu), re.IGNORECASE) is not None


def test_every_mi355x_example_pins_a_rocm7_image():
    paths = glob.glob(os.path.join(REPO, "examples", "**", "*.dstack.yml"), recursive=True) + \
        glob.glob(os.path.join(REPO, "examples", "**", ".dstack.yml"), recursive=True)
    checked = pinned = 0
    for p in paths:
        with open(p) as f:
            for conf in yaml.safe_load_all(f):
                if not isinstance(conf, dict) or not _mi35x(conf) or "image" not in conf:
                    continue
                checked += 1
                v = images.image_rocm_version(conf["image"])
                # a tag that names a ROCm names >= 7.0; AMD's PyTorch image is always pinned (third-
                # party serving images -- vLLM, TGI, Ollama -- follow their own ``latest`` ROCm builds)
                assert v is None or v >= (7, 0), f"{p}: {conf['image']} (MI355X needs ROCm >= 7.0)"
                if conf["image"].startswith("rocm/pytorch"):
                    assert v is not None, f"{p}: {conf['image']} is not pinned to a ROCm release"
                    pinned += 1
    assert checked >= 8 and pinned >= 8


def _spec(image, gpu):
    return RunSpec.model_validate({"run_name": "t", "repo_id": "r", "repo_data": {"repo_type": "virtual"},
                                   "configuration": {"type": "task", "commands": ["python train.py"],
                                                     "image": image, "resources": {"gpu": gpu}}})


def test_configurator_rejects_rocm6_image_for_mi355x_only_runs():
    old = "rocm/pytorch:rocm6.4_ubuntu22.04_py3.10_pytorch_release_2.6.0"
    with pytest.raises(ServerClientError, match=r"ROCm 6\.4.*MI355X.*ROCm >= 7\.0"):
        get_job_specs_from_run_spec(_spec(old, "MI355X:8"))
    with pytest.raises(ServerClientError):
        get_job_specs_from_run_spec(_spec(old, {"name": ["MI350X", "MI355X"], "count": 8}))
    # a run that also accepts an MI300X is valid (placement keeps it off gfx950 hosts)
    assert get_job_specs_from_run_spec(_spec(old, {"name": ["MI300X", "MI355X"], "count": 8}))
    # unnamed GPUs, a ROCm 7 image, or a tag that does not say: accepted
    assert get_job_specs_from_run_spec(_spec(old, "8"))
    assert get_job_specs_from_run_spec(_spec(images.DEFAULT_ROCM_IMAGE, "MI355X:8"))
    assert get_job_specs_from_run_spec(_spec("rocm/pytorch:latest", "MI355X:8"))


def test_placement_skips_gfx950_offers_for_rocm6_images():
    old = "rocm/pytorch:rocm6.4_ubuntu22.04_py3.10_pytorch_release_2.6.0"
    mi355 = [Gpu(name="MI355X", memory_mib=288 * 1024)] * 8
    mi300 = [Gpu(name="MI300X", memory_mib=192 * 1024)] * 8
    assert not images.offer_supported(old, mi355)
    assert images.offer_supported(old, mi300)
    assert images.offer_supported(images.DEFAULT_ROCM_IMAGE, mi355)
    assert images.offer_supported("rocm/pytorch:latest", mi355)
    assert images.offer_supported(old, [])  # CPU offers
