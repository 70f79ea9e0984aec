"""Fleets (reference: ``S/services/fleets.py:236-793``): plan, create (cloud: ``nodes`` pending
instances, optionally in a placement group; SSH: one instance per host), delete, list."""

from __future__ import annotations

import contextlib
import json
import re
import uuid
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session, object_session

from dstack_amd.core.errors import ResourceExistsError, ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import Duration
from dstack_amd.core.models.envs import Env
from dstack_amd.core.models.fleets import (
    Fleet,
    FleetConfiguration,
    FleetPlan,
    FleetSpec,
    FleetStatus,
    InstanceGroupPlacement,
    SSHHostParams,
)
from dstack_amd.core.models.instances import InstanceStatus, RemoteConnectionInfo, SSHKey
from dstack_amd.core.models.profiles import DEFAULT_FLEET_TERMINATION_IDLE_TIME, Profile
from dstack_amd.core.models.resources import ResourcesSpec
from dstack_amd.core.models.runs import JobStatus, Requirements, get_policy_map
from dstack_amd.core.models.profiles import SpotPolicy
from dstack_amd.server.background import scheduler
from dstack_amd.server.models import FleetModel, InstanceModel, ProjectModel, UserModel
from dstack_amd.server.services import offers as offers_services
from dstack_amd.server.services import pools as pools_services
from dstack_amd.server.services.locking import db_advisory_lock, lockset
from dstack_amd.server.services.permissions import check_can_manage_ssh_fleets
from dstack_amd.utils.common import generate_name, get_current_datetime


def fleet_model_to_fleet(f: FleetModel, include_terminated: bool = False) -> Fleet:
    instances = [pools_services.instance_model_to_instance(i) for i in sorted(f.instances, key=lambda i: i.instance_num)
                 if include_terminated or i.status != InstanceStatus.TERMINATED.value]
    return Fleet(id=f.id, name=f.name, project_name=f.project.name, spec=FleetSpec.model_validate_json(f.spec),
                 created_at=f.created_at, status=FleetStatus(f.status), status_message=f.status_message,
                 instances=instances)


def list_project_fleets(s: Session, project: ProjectModel) -> List[FleetModel]:
    return list(s.execute(select(FleetModel).where(FleetModel.project_id == project.id, FleetModel.deleted == False)  # noqa
                          .order_by(FleetModel.created_at)).scalars())


def get_fleet_by_name(s: Session, project: ProjectModel, name: str) -> Optional[FleetModel]:
    return s.execute(select(FleetModel).where(FleetModel.project_id == project.id, FleetModel.name == name,
                                              FleetModel.deleted == False)).scalar_one_or_none()  # noqa


def _requirements(conf: FleetConfiguration, profile: Profile) -> Requirements:
    return Requirements(resources=conf.resources or ResourcesSpec(), max_price=profile.max_price,
                        spot=get_policy_map(profile.spot_policy, SpotPolicy.ONDEMAND), reservation=profile.reservation)


def check_ssh_hosts_not_yet_added(s: Session, spec: FleetSpec, current_fleet_id=None) -> None:
    """An SSH host belongs to at most one active fleet, across every project of the server; the
    fleet being updated (``current_fleet_id``) may keep its own hosts (reference
    ``_check_ssh_hosts_not_yet_added``)."""
    sc = spec.configuration.ssh_config
    if sc is None or not sc.hosts:
        return
    existing = set()
    rows = s.execute(select(InstanceModel).where(InstanceModel.deleted == False,  # noqa: E712
                                                 InstanceModel.remote_connection_info.isnot(None),
                                                 InstanceModel.status != InstanceStatus.TERMINATED.value)).scalars()
    for inst in rows:
        if current_fleet_id is not None and inst.fleet_id == current_fleet_id:
            continue
        existing.add(RemoteConnectionInfo.model_validate_json(inst.remote_connection_info).host)
    taken = [h if isinstance(h, str) else h.hostname for h in sc.hosts
             if (h if isinstance(h, str) else h.hostname) in existing]
    if taken:
        raise ServerClientError(f"Instances [{', '.join(taken)}] are already assigned to a fleet.")


def get_plan(s: Session, project: ProjectModel, user: UserModel, spec: FleetSpec) -> FleetPlan:
    current = None
    current_id = None
    if spec.configuration.name:
        f = get_fleet_by_name(s, project, spec.configuration.name)
        current = fleet_model_to_fleet(f) if f else None
        current_id = f.id if f else None
    check_ssh_hosts_not_yet_added(s, spec, current_id)
    offers = []
    if spec.configuration.ssh_config is None:
        profile = spec.merged_profile
        offers = [o for _, o in offers_services.get_offers_by_requirements(
            s, project, profile, _requirements(spec.configuration, profile),
            multinode=spec.configuration.placement == InstanceGroupPlacement.CLUSTER,
            blocks=spec.configuration.blocks,
        )]
    return FleetPlan(project_name=project.name, user=user.name, spec=spec, current_resource=current,
                     offers=offers[:50], total_offers=len(offers), max_offer_price=max((o.price for o in offers),
                                                                                       default=None))


def _idle_seconds(conf: FleetConfiguration) -> int:
    v = conf.idle_duration
    if v is None:
        return DEFAULT_FLEET_TERMINATION_IDLE_TIME
    return int(v)


_NAME_RE = re.compile(r"^[a-z][a-z0-9-]{1,40}$")
_KEY_HEADER = re.compile(r"-----BEGIN (RSA |EC |OPENSSH )?PRIVATE KEY-----")


def _validate_fleet_spec(spec: FleetSpec):
    """Reject specs the reconcilers could never act on (reference ``_validate_fleet_spec``): a fleet
    needs ``nodes`` or ``ssh_config``; every SSH host needs a user and a usable private key (the
    CLI resolves ``identity_file`` into ``ssh_key`` on the client: the server never reads a path
    it was sent); ``internal_ip`` is given for all hosts or none, and not together with
    ``network``."""
    conf = spec.configuration
    if conf.name is not None and not _NAME_RE.match(conf.name):
        raise ServerClientError("Fleet name must be 2-41 chars of a-z, 0-9 and -, starting with a letter")
    if conf.ssh_config is None and conf.nodes is None:
        raise ServerClientError("No ssh_config or nodes specified")
    sc = conf.ssh_config
    if sc is None:
        return
    with_ip = 0
    for host in sc.hosts:
        h = host if isinstance(host, SSHHostParams) else SSHHostParams(hostname=host)
        key = h.ssh_key or sc.ssh_key
        if key is None:
            raise ServerClientError(f"No ssh key specified for host {h.hostname}")
        _validate_private_key(key)
        if (h.user or sc.user) is None:
            raise ServerClientError(f"No ssh user specified for host {h.hostname}")
        with_ip += h.internal_ip is not None
    if with_ip not in (0, len(sc.hosts)):
        raise ServerClientError("internal_ip must be specified for all hosts")
    if with_ip and sc.network is not None:
        raise ServerClientError("internal_ip is mutually exclusive with network")


def _validate_private_key(key: SSHKey):
    if not key.private:
        raise ServerClientError("Private key not provided")
    if not _KEY_HEADER.search(key.private) or "ENCRYPTED" in key.private:
        raise ServerClientError("Unsupported key type. The key type should be RSA, ECDSA, or Ed25519 and should "
                                "not be encrypted with passphrase.")


def create_fleet(s: Session, project: ProjectModel, user: UserModel, spec: FleetSpec) -> Fleet:
    conf = spec.configuration
    _validate_fleet_spec(spec)
    if conf.ssh_config is not None:
        check_can_manage_ssh_fleets(user, project)
        check_ssh_hosts_not_yet_added(s, spec)
    with db_advisory_lock(s, f"fleet_names_{project.id}"):
        if conf.name is None:
            conf.name = generate_name()
        if get_fleet_by_name(s, project, conf.name) is not None:
            raise ResourceExistsError(f"Fleet {conf.name} exists")
        fleet = FleetModel(id=uuid.uuid4(), name=conf.name, project_id=project.id, status=FleetStatus.ACTIVE.value,
                           spec=spec.model_dump_json(), created_at=get_current_datetime(),
                           last_processed_at=get_current_datetime())
        s.add(fleet)
        s.flush()
        pool = pools_services.get_or_create_default_pool(s, project)
        profile = spec.merged_profile
        if conf.ssh_config is not None:
            for i, host in enumerate(conf.ssh_config.hosts):
                h = host if isinstance(host, SSHHostParams) else SSHHostParams(hostname=host)
                user_name = h.user or conf.ssh_config.user
                port = h.port or conf.ssh_config.port or 22
                key = h.ssh_key or conf.ssh_config.ssh_key
                rci = RemoteConnectionInfo(host=h.hostname, port=port, ssh_user=user_name, ssh_keys=[key],
                                           env=conf.env)
                pools_services.create_instance_model(
                    s, project, pool, name=f"{conf.name}-{i}", status=InstanceStatus.PENDING, fleet=fleet,
                    instance_num=i, backend=BackendType.REMOTE.value, region="remote", price=0.0,
                    remote_connection_info=rci.model_dump_json(),
                    termination_idle_time=-1, termination_policy="dont-destroy",
                    total_blocks=None if h.blocks == "auto" else int(h.blocks),
                    backend_data=json.dumps({"blocks": h.blocks, "internal_ip": h.internal_ip,
                                             "network": conf.ssh_config.network}),
                )
        else:
            nodes = conf.nodes.min or 0
            for i in range(nodes):
                pools_services.create_instance_model(
                    s, project, pool, name=f"{conf.name}-{i}", status=InstanceStatus.PENDING, fleet=fleet,
                    instance_num=i, profile=profile.model_dump_json(),
                    requirements=_requirements(conf, profile).model_dump_json(),
                    termination_idle_time=_idle_seconds(conf),
                    termination_policy="destroy-after-idle" if _idle_seconds(conf) >= 0 else "dont-destroy",
                    backend_data=json.dumps({"blocks": conf.blocks,
                                             "placement": conf.placement.value if conf.placement else None}),
                )
        s.flush()
        s.refresh(fleet)
    scheduler.wake(scheduler.INSTANCES)
    return fleet_model_to_fleet(fleet)


def create_autocreated_fleet(s: Session, project: ProjectModel, run_name: str, profile: Profile,
                             multinode: bool) -> FleetModel:
    conf = FleetConfiguration(name=f"{run_name}-fleet-{uuid.uuid4().hex[:4]}", nodes=1,
                              placement=InstanceGroupPlacement.CLUSTER if multinode else None)
    spec = FleetSpec(configuration=conf, profile=profile, autocreated=True)
    fleet = FleetModel(id=uuid.uuid4(), name=conf.name, project_id=project.id, status=FleetStatus.ACTIVE.value,
                       spec=spec.model_dump_json())
    s.add(fleet)
    s.flush()
    return fleet


def _check_ssh_fleets(user, project: ProjectModel, fleets) -> None:
    if user is None:
        return
    for f in fleets:
        conf = (json.loads(f.spec or "{}") or {}).get("configuration") or {}
        if conf.get("ssh_config") is not None:
            check_can_manage_ssh_fleets(user, project)


def delete_fleets(s: Session, project: ProjectModel, names: List[str], user: Optional[UserModel] = None):
    """Fleets and their instances are held in the background processors' locksets while their
    state is re-read, checked and changed, and committed before release: a job assigned to an
    instance (IDLE -> BUSY) or an instance pass (PROVISIONING -> IDLE) racing the delete can then
    neither slip past the busy check nor write over TERMINATING."""
    fleets = []
    for name in names:
        f = get_fleet_by_name(s, project, name)
        if f is None:
            raise ResourceNotExistsError(f"Fleet {name} not found")
        fleets.append(f)
    _check_ssh_fleets(user, project, fleets)
    for _attempt in range(5):
        locked = [i for f in fleets for i in f.instances]
        with _held(fleets, locked):
            for f in fleets:
                s.refresh(f, ["instances"])  # instances added since the lock set was built
            if {i.id for f in fleets for i in f.instances} != {i.id for i in locked}:
                s.rollback()
                continue  # an instance joined a fleet meanwhile: lock the new set and re-check
            _terminate_fleets_locked(s, fleets)
            s.commit()
            break
    else:
        from dstack_amd.core.errors import ResourceBusyError

        raise ResourceBusyError("Fleet instances keep changing, retry")
    scheduler.wake(scheduler.INSTANCES, scheduler.FLEETS)


def _instance_in_use(inst) -> bool:
    """BUSY, or holding a job that is not finished (e.g. PROVISIONING for a just-submitted job)."""
    if inst.status == InstanceStatus.BUSY.value:
        return True
    return any(not JobStatus(j.status).is_finished() for j in inst.jobs)


def _terminate_fleets_locked(s: Session, fleets):
    for f in fleets:
        busy = [i for i in f.instances if _instance_in_use(i)]
        if busy:
            raise ServerClientError(f"Fleet {f.name} has busy instances; stop the runs first")
    for f in fleets:
        for inst in f.instances:
            if inst.status not in (InstanceStatus.TERMINATING.value, InstanceStatus.TERMINATED.value):
                inst.status = InstanceStatus.TERMINATING.value
                inst.termination_reason = "fleet deleted"
        f.status = FleetStatus.TERMINATING.value


def delete_fleet_instances(s: Session, project: ProjectModel, name: str, instance_nums: List[int],
                           user: Optional[UserModel] = None):
    f = get_fleet_by_name(s, project, name)
    if f is None:
        raise ResourceNotExistsError(f"Fleet {name} not found")
    _check_ssh_fleets(user, project, [f])
    targets = [i for i in f.instances if i.instance_num in instance_nums]
    with _held([], targets):
        for inst in targets:
            if _instance_in_use(inst):
                raise ServerClientError(f"Instance {inst.name} is busy")
        for inst in targets:
            inst.status = InstanceStatus.TERMINATING.value
            inst.termination_reason = "deleted by user"
        s.commit()
    scheduler.wake(scheduler.INSTANCES)


@contextlib.contextmanager
def _held(fleets, instances, timeout: float = 60.0):
    """Hold fleets and instances in their background locksets and re-read them (row-locked on
    Postgres) so the block sees the state the last background pass committed."""
    with lockset("fleets").hold([f.id for f in fleets], timeout), \
            lockset("instances").hold([i.id for i in instances], timeout):
        for obj in [*fleets, *instances]:
            sess = object_session(obj)
            sess.refresh(obj, with_for_update=True)
        yield


def create_instance(s: Session, project: ProjectModel, user: UserModel, profile: Profile,
                    requirements: Requirements) -> Instance:
    """Legacy ``runs/create_instance`` (reference: ``S/services/fleets.py`` create_instance): one
    PENDING cloud instance in an auto-created fleet; the instance reconciler provisions it from
    the offers matching ``requirements``."""
    from dstack_amd.core.models.backends import BACKENDS_WITH_CREATE_INSTANCE_SUPPORT

    offers = offers_services.get_offers_by_requirements(s, project, profile, requirements,
                                                        exclude_not_available=True)
    offers = [(c, o) for c, o in offers
              if o.backend in BACKENDS_WITH_CREATE_INSTANCE_SUPPORT and o.backend != BackendType.REMOTE]
    if not offers:
        raise ServerClientError("Backends do not support create_instance or have no offers for the requirements. "
                                "Try to select other backends.")
    best = offers[0][1]
    pool = pools_services.get_or_create_pool_by_name(s, project, profile.pool_name)
    name = f"{profile.name or 'instance'}-{uuid.uuid4().hex[:6]}"
    fleet = create_autocreated_fleet(s, project, name, profile, multinode=False)
    inst = pools_services.create_instance_model(
        s, project, pool, name=f"{fleet.name}-0", status=InstanceStatus.PENDING, fleet=fleet, instance_num=0,
        profile=profile.model_dump_json(), requirements=requirements.model_dump_json(),
        termination_idle_time=DEFAULT_FLEET_TERMINATION_IDLE_TIME, termination_policy="destroy-after-idle",
        backend_data=json.dumps({"blocks": 1, "placement": None}),
        # the best offer now; the reconciler provisions from the current offers in the same order
        backend=best.backend.value, region=best.region, price=best.price, offer=best.model_dump_json(),
    )
    s.flush()
    scheduler.wake(scheduler.INSTANCES)
    return pools_services.instance_model_to_instance(inst)
