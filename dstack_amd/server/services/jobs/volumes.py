"""Network volumes of a job: resolution, attach checks, attach on provisioning, detach on
termination (reference: ``get_job_configured_volumes`` / ``check_can_attach_job_volumes``
``S/services/jobs/__init__.py:551-640``, the attach step of ``process_submitted_jobs.py:418-490``,
``process_volumes_detaching`` ``S/services/jobs/__init__.py:304-334`` and
``_should_force_detach_volume`` ``:524-536``).

A mount point names one volume or a list of alternatives (``name: [vol-us, vol-eu]``); after
``${{ dstack.node_rank }}`` interpolation (done by the job configurator) the alternatives are
resolved to ACTIVE volumes, and the one matching the instance's backend/region is attached.  The
shim receives ``{name, backend, volume_id, device_name, init_fs}`` per attached volume and mounts it
under ``/dstack-volumes/<name>`` (``native/shim/volumes.cpp``).
"""

from __future__ import annotations

import logging
from datetime import timedelta
from typing import Iterable, List, Optional, Sequence, Tuple

from sqlalchemy import delete, insert, select, update
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ComputeError, ResourceBusyError, ServerClientError
from dstack_amd.core.models.backends import BACKENDS_WITH_VOLUMES_SUPPORT, BackendType
from dstack_amd.core.models.runs import JobSpec
from dstack_amd.core.models.volumes import (
    VolumeAttachmentData,
    VolumeMountPoint,
    VolumeProvisioningData,
    VolumeStatus,
)
from dstack_amd.server.models import InstanceModel, JobModel, ProjectModel, VolumeModel, volumes_attachments
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)

# a volume that is still attached this long after the job's stop is force-detached (reference
# ``_should_force_detach_volume``: stop_duration + a grace period)
FORCE_DETACH_GRACE = timedelta(seconds=60)


def volume_mount_points(spec: JobSpec) -> List[VolumeMountPoint]:
    return [mp for mp in spec.mount_points() if isinstance(mp, VolumeMountPoint)]


def get_job_configured_volumes(s: Session, project: ProjectModel, spec: JobSpec) -> List[List[VolumeModel]]:
    """One list of candidate volumes per mount point; raises when a name does not exist."""
    from dstack_amd.server.services.volumes import get_volume_by_name

    out: List[List[VolumeModel]] = []
    for mp in volume_mount_points(spec):
        names = [mp.name] if isinstance(mp.name, str) else list(mp.name)
        cands = []
        for n in names:
            v = get_volume_by_name(s, project, n)
            if v is None:
                raise ServerClientError(f"Volume {n} not found")
            cands.append(v)
        out.append(cands)
    return out


def _vpd(v: VolumeModel) -> Optional[VolumeProvisioningData]:
    return VolumeProvisioningData.model_validate_json(v.volume_provisioning_data) \
        if v.volume_provisioning_data else None


def _backend_region(v: VolumeModel) -> Tuple[BackendType, str]:
    from dstack_amd.core.models.volumes import VolumeConfiguration

    conf = VolumeConfiguration.model_validate_json(v.configuration)
    return conf.backend, conf.region


def check_can_attach_job_volumes(volumes: Sequence[Sequence[VolumeModel]]):
    """All candidates must be ACTIVE and attachable; a mount point's alternatives must be in
    different backend/regions (else the choice would be ambiguous), and every mount point of a job
    must have an alternative in each backend/region another mount point can use."""
    for cands in volumes:
        seen = set()
        for v in cands:
            if v.status != VolumeStatus.ACTIVE.value:
                raise ServerClientError(f"Volume {v.name} is not active (status: {v.status})")
            vpd = _vpd(v)
            if vpd is not None and not vpd.attachable:
                raise ServerClientError(f"Volume {v.name} cannot be attached")
            br = _backend_region(v)
            if br in seen:
                raise ServerClientError(f"Volume alternatives {[x.name for x in cands]} share backend/region {br}")
            seen.add(br)
            if br[0] not in BACKENDS_WITH_VOLUMES_SUPPORT:
                raise ServerClientError(f"Backend {br[0].value} does not support volumes")
    names = [v.name for cands in volumes for v in cands]
    if len(names) != len(set(names)):
        raise ServerClientError("Cannot attach the same volume at different mount points")
    if len(volumes) > 1:
        common = set.intersection(*({_backend_region(v) for v in cands} for cands in volumes))
        if not common:
            raise ServerClientError("Volumes of the run have no backend/region in common")


def allowed_locations(volumes: Sequence[Sequence[VolumeModel]]) -> Optional[set]:
    """{(backend, region)} every mount point can be satisfied in; ``None`` = unconstrained."""
    if not volumes:
        return None
    return set.intersection(*({_backend_region(v) for v in cands} for cands in volumes))


def filter_offers_by_volumes(offers: Iterable, volumes: Sequence[Sequence[VolumeModel]]) -> list:
    locs = allowed_locations(volumes)
    if locs is None:
        return list(offers)
    return [(c, o) for c, o in offers if (o.backend, o.region) in locs]


def instance_matches_volumes(inst: InstanceModel, volumes: Sequence[Sequence[VolumeModel]]) -> bool:
    locs = allowed_locations(volumes)
    if locs is None:
        return True
    try:
        return (BackendType(inst.backend), inst.region) in locs
    except ValueError:
        return False


def _attached_instance_ids(s: Session, v: VolumeModel) -> List:
    return list(s.execute(select(volumes_attachments.c.instance_id)
                          .where(volumes_attachments.c.volume_id == v.id)).scalars())


def _hold_volume(s: Session, v: VolumeModel, timeout: float = 1.0):
    """Hold ``v`` in the volumes lockset until ``s`` commits, then re-read it: a concurrent
    ``delete_volumes`` (which holds the same lock and commits inside) either finishes first, and the
    attach sees ``deleted``, or waits and sees the attachment.  Contention (another job's attach
    transaction still holds the volume, e.g. while it talks to its shim) raises
    ``ResourceBusyError``: the caller retries on its next pass, the job does not fail."""
    import time

    from dstack_amd.server.services.locking import lockset, release_at_transaction_end

    held = s.info.get("held_volumes")
    if held is None:  # volumes this transaction holds; forgotten when it ends (the locks go too)
        from sqlalchemy import event

        held = s.info["held_volumes"] = set()
        for name in ("after_commit", "after_rollback"):
            event.listen(s, name, lambda _s: s.info.pop("held_volumes", None), once=True)
    if v.id not in held:
        ls = lockset("volumes")
        deadline = time.monotonic() + timeout
        while not ls.add_all_or_nothing([v.id]):
            if time.monotonic() > deadline:
                raise ResourceBusyError(f"Volume {v.name} is busy")
            time.sleep(0.005)
        held.add(v.id)
        release_at_transaction_end(s, ls, [v.id])
    s.refresh(v, with_for_update=True)


def attach_job_volumes(s: Session, job: JobModel, inst: InstanceModel,
                       volumes: Sequence[Sequence[VolumeModel]]) -> List[str]:
    """Attach the matching alternative of every mount point to ``inst``; returns the attached
    volume names (stored in ``JobRuntimeData.volume_names``).  A volume already attached to another
    instance fails the job (single-attach block storage)."""
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services.jobs import job_jpd
    from dstack_amd.server.services.volumes import volume_model_to_volume

    names = []
    jpd = job_jpd(job)
    backend = BackendType(inst.backend)
    for cands in volumes:
        v = next((x for x in cands if _backend_region(x) == (backend, inst.region)), None)
        if v is None:
            raise ServerClientError(f"No volume among {[x.name for x in cands]} in {backend.value}/{inst.region}")
        _hold_volume(s, v)
        if v.deleted:
            raise ServerClientError(f"Volume {v.name} was deleted")
        attached = _attached_instance_ids(s, v)
        if inst.id in attached:
            names.append(v.name)
            continue
        if attached:
            raise ServerClientError(f"Volume {v.name} is attached to another instance")
        compute = backends_services.get_project_backend(s, job.run.project, backend)
        instance_id = jpd.instance_id if jpd is not None else str(inst.id)
        try:
            vad = compute.attach_volume(volume_model_to_volume(v), instance_id)
        except NotImplementedError:
            vad = VolumeAttachmentData()
        except ComputeError as e:
            raise ServerClientError(f"Failed to attach volume {v.name}: {e}") from e
        s.execute(insert(volumes_attachments).values(volume_id=v.id, instance_id=inst.id,
                                                      attachment_data=vad.model_dump_json()))
        v.volume_attachment_data = vad.model_dump_json()
        names.append(v.name)
    return names


def shim_volume_specs(s: Session, job: JobModel, volume_names: Optional[List[str]]) -> List[dict]:
    """The ``volumes`` field of the shim's task body."""
    from dstack_amd.server.services.volumes import get_volume_by_name

    out = []
    for n in volume_names or []:
        v = get_volume_by_name(s, job.run.project, n)
        if v is None:
            continue
        vpd = _vpd(v)
        vad = VolumeAttachmentData.model_validate_json(v.volume_attachment_data) if v.volume_attachment_data else None
        backend, _ = _backend_region(v)
        out.append({
            "backend": backend.value, "name": v.name, "volume_id": vpd.volume_id if vpd else "",
            "device_name": (vad.device_name if vad else None) or "",
            # volumes created by dstack start empty: the shim makes a filesystem when none exists;
            # registered (external) volumes are never formatted
            "init_fs": not bool(_volume_conf_external(v)),
        })
    return out


def _volume_conf_external(v: VolumeModel) -> bool:
    from dstack_amd.core.models.volumes import VolumeConfiguration

    return VolumeConfiguration.model_validate_json(v.configuration).volume_id is not None


def detach_job_volumes(s: Session, job: JobModel, instance_id_model, stopped_at) -> bool:
    """Detach the job's volumes from its instance; ``True`` once all are detached.  Soft detach
    first; after ``stop_duration`` + grace a still-attached volume is force-detached."""
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services.jobs import job_jpd, job_jrd, job_spec
    from dstack_amd.server.services.volumes import get_volume_by_name, volume_model_to_volume

    jrd = job_jrd(job)
    names = (jrd.volume_names if jrd else None) or []
    if not names:
        return True
    jpd = job_jpd(job)
    inst = s.get(InstanceModel, instance_id_model) if instance_id_model is not None else None
    if inst is None:
        return True
    # another job on the same (shared) instance that still runs keeps the volume mounted
    others = [j for j in inst.jobs if j.id != job.id and j.status in ("provisioning", "pulling", "running")]
    in_use = {n for j in others for n in ((job_jrd(j).volume_names or []) if job_jrd(j) else [])}
    spec = job_spec(job)
    force = stopped_at is not None and get_current_datetime() - stopped_at > \
        timedelta(seconds=int(spec.stop_duration or 0)) + FORCE_DETACH_GRACE
    all_done = True
    for n in names:
        if n in in_use:
            continue
        v = get_volume_by_name(s, job.run.project, n)
        if v is None or inst.id not in _attached_instance_ids(s, v):
            continue
        backend, _ = _backend_region(v)
        compute = backends_services.get_project_backend(s, job.run.project, backend)
        vol = volume_model_to_volume(v)
        instance_id = jpd.instance_id if jpd is not None else str(inst.id)
        try:
            compute.detach_volume(vol, instance_id, force=force)
            detached = compute.is_volume_detached(vol, instance_id)
        except NotImplementedError:
            detached = True
        except ComputeError as e:
            logger.warning("detach %s from %s failed: %s", n, instance_id, e)
            detached = False
        if detached:
            s.execute(delete(volumes_attachments).where(volumes_attachments.c.volume_id == v.id,
                                                        volumes_attachments.c.instance_id == inst.id))
            s.execute(update(VolumeModel).where(VolumeModel.id == v.id).values(volume_attachment_data=None))
        else:
            all_done = False
    return all_done
