"""Offer selection (reference: ``S/services/offers.py:24-162``): backend/region restrictions for
multinode, privileged, instance mounts, reservations and the master job."""

from __future__ import annotations

from typing import List, Optional, Tuple

from sqlalchemy.orm import Session

from dstack_amd.core.backends.base import Compute
from dstack_amd.core.models.backends import (
    BACKENDS_WITH_INSTANCE_VOLUMES_SUPPORT,
    BACKENDS_WITH_MULTINODE_SUPPORT,
    BACKENDS_WITH_PRIVILEGED_SUPPORT,
    BACKENDS_WITH_RESERVATION_SUPPORT,
    BackendType,
)
from dstack_amd.core.models.instances import InstanceOfferWithAvailability
from dstack_amd.core.models.profiles import Profile
from dstack_amd.core.models.runs import JobProvisioningData, Requirements
from dstack_amd.server.models import ProjectModel
from dstack_amd.server.services import backends as backends_services


def get_offers_by_requirements(
    s: Session, project: ProjectModel, profile: Profile, requirements: Requirements,
    exclude_not_available: bool = False, multinode: bool = False,
    master_job_provisioning_data: Optional[JobProvisioningData] = None, privileged: bool = False,
    instance_mounts: bool = False, blocks: int = 1,
) -> List[Tuple[Compute, InstanceOfferWithAvailability]]:
    backends = backends_services.get_project_backends(s, project)
    backend_types = profile.backends
    regions = profile.regions
    if multinode:
        backend_types = [b for b in (backend_types or [t for t, _ in backends]) if b in BACKENDS_WITH_MULTINODE_SUPPORT]
    if privileged:
        backend_types = [b for b in (backend_types or [t for t, _ in backends]) if b in BACKENDS_WITH_PRIVILEGED_SUPPORT]
    if instance_mounts:
        backend_types = [b for b in (backend_types or [t for t, _ in backends])
                         if b in BACKENDS_WITH_INSTANCE_VOLUMES_SUPPORT]
    if profile.reservation:
        backend_types = [b for b in (backend_types or [t for t, _ in backends]) if b in BACKENDS_WITH_RESERVATION_SUPPORT]
    if master_job_provisioning_data is not None:
        backend_types = [master_job_provisioning_data.get_base_backend()]
        regions = [master_job_provisioning_data.region]
    if backend_types is not None:
        backends = [(t, c) for t, c in backends if t in backend_types]
    offers = backends_services.get_instance_offers(backends, requirements, exclude_not_available)
    if regions:
        offers = [(c, o) for c, o in offers if o.region in regions or o.backend == BackendType.LOCAL]
    if profile.instance_types:
        names = {n.lower() for n in profile.instance_types}
        offers = [(c, o) for c, o in offers if o.instance.name.lower() in names]
    if blocks != 1:
        offers = [(c, _with_blocks(o, blocks)) for c, o in offers if _divisible(o, blocks)]
    return offers


def _divisible(offer: InstanceOfferWithAvailability, blocks) -> bool:
    if blocks == "auto":
        return True
    n = len(offer.instance.resources.gpus)
    return (n == 0 or n % blocks == 0) and offer.instance.resources.cpus % blocks == 0


def _with_blocks(offer: InstanceOfferWithAvailability, blocks) -> InstanceOfferWithAvailability:
    from dstack_amd.core.backends.remote import auto_blocks

    res = offer.instance.resources
    total = auto_blocks(len(res.gpus), res.cpus) if blocks == "auto" else blocks
    return offer.model_copy(update={"total_blocks": total})
