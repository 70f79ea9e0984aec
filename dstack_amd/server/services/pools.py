"""Pools and pool instances (reference: ``S/services/pools.py:409-797``): instance model
conversion, reuse filtering, shared (block) offers, instance creation."""

from __future__ import annotations

import json
import uuid
from typing import List, Optional, Tuple

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.backends.base import offer_matches
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.fleets import Instance
from dstack_amd.core.models.instances import (
    Disk,
    Gpu,
    HostTopology,
    InstanceAvailability,
    InstanceOfferWithAvailability,
    InstanceStatus,
    InstanceType,
    Resources,
)
from dstack_amd.core.models.profiles import DEFAULT_POOL_NAME, Profile
from dstack_amd.core.models.runs import JobProvisioningData, Requirements
from dstack_amd.server.models import FleetModel, InstanceModel, PoolModel, ProjectModel
from dstack_amd.utils.common import get_current_datetime


def get_or_create_default_pool(s: Session, project: ProjectModel) -> PoolModel:
    pool = s.execute(select(PoolModel).where(PoolModel.project_id == project.id, PoolModel.name == DEFAULT_POOL_NAME,
                                             PoolModel.deleted == False)).scalar_one_or_none()  # noqa: E712
    if pool is None:
        pool = PoolModel(id=uuid.uuid4(), name=DEFAULT_POOL_NAME, project_id=project.id)
        s.add(pool)
        s.flush()
        project.default_pool_id = pool.id
    return pool


def instance_offer(inst: InstanceModel) -> Optional[InstanceOfferWithAvailability]:
    return InstanceOfferWithAvailability.model_validate_json(inst.offer) if inst.offer else None


def instance_jpd(inst: InstanceModel) -> Optional[JobProvisioningData]:
    return JobProvisioningData.model_validate_json(inst.job_provisioning_data) if inst.job_provisioning_data else None


def instance_topology(inst: InstanceModel) -> Optional[HostTopology]:
    return HostTopology.model_validate_json(inst.host_topology) if inst.host_topology else None


def instance_model_to_instance(inst: InstanceModel) -> Instance:
    offer = instance_offer(inst)
    jpd = instance_jpd(inst)
    health = json.loads(inst.health_data) if inst.health_data else None
    return Instance(
        id=inst.id, project_name=inst.project.name if inst.project else "", backend=BackendType(inst.backend)
        if inst.backend else None, instance_type=jpd.instance_type if jpd else (offer.instance if offer else None),
        name=inst.name, fleet_id=inst.fleet_id, fleet_name=inst.fleet.name if inst.fleet else None,
        instance_num=inst.instance_num, pool_name=inst.pool.name if inst.pool else None,
        hostname=jpd.hostname if jpd else None, status=InstanceStatus(inst.status), unreachable=inst.unreachable,
        termination_reason=inst.termination_reason, created=inst.created_at, region=inst.region, price=inst.price,
        total_blocks=inst.total_blocks, busy_blocks=inst.busy_blocks, health=health,
    )


def list_project_instances(s: Session, project: ProjectModel, include_terminated: bool = False) -> List[InstanceModel]:
    q = select(InstanceModel).where(InstanceModel.project_id == project.id, InstanceModel.deleted == False)  # noqa
    rows = list(s.execute(q.order_by(InstanceModel.created_at)).scalars())
    if not include_terminated:
        rows = [r for r in rows if r.status != InstanceStatus.TERMINATED.value]
    return rows


def _scaled_resources(res: Resources, blocks: int, total_blocks: int) -> Resources:
    if total_blocks <= 1:
        return res
    n = len(res.gpus)
    gpus = res.gpus[: n * blocks // total_blocks] if n else []
    return Resources(cpus=res.cpus * blocks // total_blocks, memory_mib=res.memory_mib * blocks // total_blocks,
                     gpus=gpus, spot=res.spot, disk=Disk(size_mib=res.disk.size_mib * blocks // total_blocks),
                     description=res.description)


def generate_shared_offer(offer: InstanceOfferWithAvailability, blocks: int, total_blocks: int):
    return InstanceOfferWithAvailability(
        backend=offer.backend, instance=InstanceType(name=offer.instance.name,
                                                     resources=_scaled_resources(offer.instance.resources, blocks,
                                                                                 total_blocks)),
        region=offer.region, price=offer.price * blocks / max(1, total_blocks), availability=offer.availability,
        instance_runtime=offer.instance_runtime, blocks=blocks, total_blocks=total_blocks,
    )


def get_instance_shared_offer(inst: InstanceModel, requirements: Requirements) -> Optional[InstanceOfferWithAvailability]:
    """Smallest number of free blocks of ``inst`` that satisfies the requirements
    (``is_divisible_into_blocks`` + ``get_shared_pool_instances_with_offers``)."""
    offer = instance_offer(inst)
    if offer is None:
        return None
    total = inst.total_blocks or 1
    free = total - (inst.busy_blocks or 0)
    if free <= 0:
        return None
    for blocks in range(1, free + 1):
        if total % blocks != 0 and blocks != free:
            continue
        shared = generate_shared_offer(offer, blocks, total)
        # an instance offer always matches its own host: ignore disk lower bound
        req = requirements.model_copy(deep=True)
        req.resources.disk = None
        if offer_matches(shared, req):
            avail = InstanceAvailability.IDLE if inst.status == InstanceStatus.IDLE.value else InstanceAvailability.BUSY
            shared.availability = avail
            return shared
    return None


def filter_pool_instances(
    instances: List[InstanceModel], profile: Profile, requirements: Requirements,
    fleet: Optional[FleetModel] = None, multinode: bool = False, master_jpd: Optional[JobProvisioningData] = None,
) -> List[Tuple[InstanceModel, InstanceOfferWithAvailability]]:
    out = []
    for inst in instances:
        if inst.status not in (InstanceStatus.IDLE.value, InstanceStatus.BUSY.value) or inst.unreachable:
            continue
        if inst.health_data and not json.loads(inst.health_data).get("healthy", True):
            continue  # its GPUs failed the HIP health probe (HBM/MFMA below thresholds)
        if fleet is not None and inst.fleet_id != fleet.id:
            continue
        if profile.backends and inst.backend and BackendType(inst.backend) not in profile.backends:
            continue
        if profile.regions and inst.region and inst.region not in profile.regions:
            continue
        if profile.instance_types:
            off = instance_offer(inst)
            if off and off.instance.name not in profile.instance_types:
                continue
        if multinode and (inst.total_blocks or 1) > 1 and (inst.busy_blocks or 0) > 0:
            continue  # multinode jobs never share an instance
        if master_jpd is not None:
            jpd = instance_jpd(inst)
            if jpd and (jpd.backend != master_jpd.backend or jpd.region != master_jpd.region):
                continue
        shared = get_instance_shared_offer(inst, requirements)
        if shared is not None:
            if multinode and shared.blocks != (inst.total_blocks or 1):
                shared = generate_shared_offer(instance_offer(inst), inst.total_blocks or 1, inst.total_blocks or 1)
                if (inst.busy_blocks or 0) > 0:
                    continue
            out.append((inst, shared))
    out.sort(key=lambda t: (t[0].status != InstanceStatus.IDLE.value, t[1].price, t[0].created_at))
    return out


def create_instance_model(s: Session, project: ProjectModel, pool: PoolModel, name: str, status: InstanceStatus,
                          fleet: Optional[FleetModel] = None, instance_num: int = 0, **kw) -> InstanceModel:
    inst = InstanceModel(id=uuid.uuid4(), name=name, instance_num=instance_num, project_id=project.id,
                         pool_id=pool.id, fleet_id=fleet.id if fleet else None, status=status.value,
                         unreachable=False, created_at=get_current_datetime(), last_processed_at=get_current_datetime(),
                         busy_gpus="", **kw)
    s.add(inst)
    s.flush()
    return inst


# ---- legacy pool API (reference: S/services/pools.py:64-380, routers/pools.py; deprecated there) --
def get_pool(s: Session, project: ProjectModel, name: str) -> Optional[PoolModel]:
    return s.execute(select(PoolModel).where(PoolModel.project_id == project.id, PoolModel.name == name,
                                             PoolModel.deleted == False)).scalar_one_or_none()  # noqa: E712


def get_or_create_pool_by_name(s: Session, project: ProjectModel, name: Optional[str]) -> PoolModel:
    if name is None:
        if project.default_pool_id is not None:
            pool = s.get(PoolModel, project.default_pool_id)
            if pool is not None and not pool.deleted:
                return pool
        return get_or_create_default_pool(s, project)
    pool = get_pool(s, project, name)
    if pool is None:
        pool = create_pool(s, project, name)
    return pool


def _pool_instances(pool: PoolModel) -> List[InstanceModel]:
    return [i for i in pool.instances if not i.deleted]


def pool_model_to_pool(project: ProjectModel, pool: PoolModel):
    from dstack_amd.core.models.fleets import Pool

    insts = _pool_instances(pool)
    avail = sum(1 for i in insts if i.status in (InstanceStatus.IDLE.value, InstanceStatus.BUSY.value))
    return Pool(name=pool.name, default=project.default_pool_id == pool.id, created_at=pool.created_at,
                total_instances=len(insts), available_instances=avail)


def generate_instance_name(s: Session, project: ProjectModel, pool_name: Optional[str]) -> str:
    """A random ``adjective-noun`` name not yet used by a live instance of the pool (reference:
    ``S/services/pools.py`` ``generate_instance_name``)."""
    from dstack_amd.utils.common import generate_name

    pool = get_or_create_pool_by_name(s, project, pool_name)
    taken = {i.name for i in _pool_instances(pool)}
    name = generate_name()
    for _ in range(64):
        if name not in taken:
            return name
        name = generate_name()
    n = 1
    while f"{name}-{n}" in taken:
        n += 1
    return f"{name}-{n}"


def list_project_pools(s: Session, project: ProjectModel):
    pools = list(s.execute(select(PoolModel).where(PoolModel.project_id == project.id,
                                                   PoolModel.deleted == False)).scalars())  # noqa: E712
    if not pools:
        pools = [get_or_create_default_pool(s, project)]
    return [pool_model_to_pool(project, p) for p in pools]


def create_pool(s: Session, project: ProjectModel, name: str) -> PoolModel:
    from dstack_amd.core.errors import ResourceExistsError

    if get_pool(s, project, name) is not None:
        raise ResourceExistsError(f"Pool {name} exists")
    pool = PoolModel(id=uuid.uuid4(), name=name, project_id=project.id)
    s.add(pool)
    s.flush()
    if project.default_pool_id is None:
        project.default_pool_id = pool.id
    return pool


def set_default_pool(s: Session, project: ProjectModel, name: str):
    from dstack_amd.core.errors import ResourceNotExistsError

    pool = get_pool(s, project, name)
    if pool is None:
        raise ResourceNotExistsError("Pool not found")
    project.default_pool_id = pool.id


def delete_pool(s: Session, project: ProjectModel, name: str):
    from dstack_amd.core.errors import ResourceNotExistsError, ServerClientError

    pool = get_pool(s, project, name)
    if pool is None:
        raise ResourceNotExistsError("Pool not found")
    if any(i.status != InstanceStatus.TERMINATED.value for i in _pool_instances(pool)):
        raise ServerClientError("Cannot delete pool with running instances")
    pool.deleted = True
    pool.deleted_at = get_current_datetime()
    if project.default_pool_id == pool.id:
        project.default_pool_id = None


def remove_instance(s: Session, project: ProjectModel, pool_name: str, instance_name: str, force: bool):
    """Mark a pool instance for termination (an instance running jobs only with ``force``)."""
    from dstack_amd.core.errors import ResourceNotExistsError
    from dstack_amd.server.background import scheduler

    pool = get_pool(s, project, pool_name)
    if pool is None:
        raise ResourceNotExistsError("Pool not found")
    from dstack_amd.server.services.locking import lockset

    named = [i for i in _pool_instances(pool) if i.name == instance_name]
    done = False
    # held in the instances lockset and committed inside, like the fleet deletes: a job assigned
    # to the instance meanwhile (its lock is kept until that assignment commits) is seen here
    with lockset("instances").hold([i.id for i in named], timeout=60.0):
        for inst in named:
            s.refresh(inst, with_for_update=True)
            if force or not inst.jobs:
                inst.status = InstanceStatus.TERMINATING.value
                done = True
        if not done:
            raise ResourceNotExistsError("Could not find instance to terminate")
        s.commit()
    scheduler.wake(scheduler.INSTANCES)


def show_pool_instances(s: Session, project: ProjectModel, name: Optional[str]):
    from dstack_amd.core.errors import ResourceNotExistsError
    from dstack_amd.core.models.fleets import PoolInstances

    if name is not None:
        pool = get_pool(s, project, name)
        if pool is None:
            raise ResourceNotExistsError("Pool not found")
    else:
        pool = get_or_create_pool_by_name(s, project, None)
    return PoolInstances(name=pool.name, instances=[instance_model_to_instance(i) for i in _pool_instances(pool)])


def add_remote(s: Session, project: ProjectModel, pool_name: Optional[str], instance_name: Optional[str],
               instance_network: Optional[str], region: Optional[str], host: str, port: int, ssh_user: str,
               ssh_keys) -> Instance:
    """Register an SSH host as a pool instance (PENDING -> the instance reconciler deploys the shim
    and reads back host_info, exactly as for SSH-fleet hosts).  Idempotent per host/port/user."""
    import ipaddress

    from dstack_amd.core.errors import ServerClientError
    from dstack_amd.core.models.instances import RemoteConnectionInfo
    from dstack_amd.server.background import scheduler

    if instance_network is not None:
        try:
            instance_network = str(ipaddress.IPv4Interface(instance_network).network)
        except ValueError:
            raise ServerClientError("Failed to parse network value")
    insts = s.execute(select(InstanceModel).where(InstanceModel.project_id == project.id,
                                                  InstanceModel.deleted == False)).scalars()  # noqa: E712
    for inst in insts:
        if inst.remote_connection_info:
            rci = RemoteConnectionInfo.model_validate_json(inst.remote_connection_info)
            if rci.host == host and rci.port == port and rci.ssh_user == ssh_user:
                return instance_model_to_instance(inst)
    pool = get_or_create_pool_by_name(s, project, pool_name)
    if instance_name is None:
        instance_name = generate_instance_name(s, project, pool.name)
    rci = RemoteConnectionInfo(host=host, port=port, ssh_user=ssh_user, ssh_keys=ssh_keys)
    inst = create_instance_model(
        s, project, pool, name=instance_name, status=InstanceStatus.PENDING, backend=BackendType.REMOTE.value,
        region=region or "remote", price=0.0, remote_connection_info=rci.model_dump_json(),
        termination_idle_time=-1, termination_policy="dont-destroy",
        backend_data=json.dumps({"blocks": 1, "internal_ip": None, "network": instance_network}),
    )
    s.flush()
    scheduler.wake(scheduler.INSTANCES)
    return instance_model_to_instance(inst)
