"""Instance lifecycle (reference: ``S/background/tasks/process_instances.py:112-965``).

PENDING: SSH-fleet hosts are deployed (shim + runner over ssh/scp, host_info with the amdsmi/xGMI
topology); cloud-fleet instances are created through the backends.  PROVISIONING: wait for the
hostname, then the shim healthcheck -> IDLE.  IDLE/BUSY: shim healthcheck (unreachable hosts are
terminated after 20 min), idle-duration expiry -> TERMINATING.  TERMINATING: backend terminate.
"""

from __future__ import annotations

import json
import logging
import uuid
from datetime import timedelta
from typing import Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.backends.remote import (
    auto_blocks,
    deploy_ssh_instance,
    host_info_to_instance_type,
    remote_backend_data,
    split_blocks,
)
from dstack_amd.core.errors import ProvisioningError
from dstack_amd.core.models.backends import BACKENDS_WITH_CREATE_INSTANCE_SUPPORT, BACKENDS_WITH_PLACEMENT_GROUPS_SUPPORT, BackendType
from dstack_amd.core.models.fleets import InstanceGroupPlacement
from dstack_amd.core.models.instances import (
    InstanceAvailability,
    InstanceConfiguration,
    InstanceOfferWithAvailability,
    InstanceStatus,
    RemoteConnectionInfo,
    SSHKey,
)
from dstack_amd.core.models.profiles import Profile, RetryEvent
from dstack_amd.core.models.runs import JobProvisioningData, Requirements
from dstack_amd.server.background import scheduler
from dstack_amd.server.background.common import claim_and_process
from dstack_amd.server.models import InstanceModel
from dstack_amd.server.services import backends as backends_services
from dstack_amd.server.services import offers as offers_services
from dstack_amd.server.services import pools as pools_services
from dstack_amd.server.services.runner.client import get_shim_client
from dstack_amd.utils.common import get_current_datetime, get_ip_from_network

logger = logging.getLogger(__name__)

TERMINATION_DEADLINE_OFFSET = timedelta(minutes=20)
PROVISIONING_DEADLINE = timedelta(minutes=20)
SSH_DEPLOY_RETRY = timedelta(seconds=30)


def process_instances(batch: int = 5) -> bool:
    def select_ids(s: Session):
        return s.execute(select(InstanceModel.id).where(InstanceModel.status != InstanceStatus.TERMINATED.value)
                         .where(InstanceModel.deleted == False)  # noqa: E712
                         .order_by(InstanceModel.last_processed_at).limit(batch * 4)).scalars()

    return claim_and_process("instances", select_ids, _process_instance, batch)


def _process_instance(s: Session, inst_id):
    inst = s.get(InstanceModel, inst_id)
    if inst is None:
        return
    st = InstanceStatus(inst.status)
    if st == InstanceStatus.PENDING:
        if inst.remote_connection_info:
            _add_remote(s, inst)
        else:
            _create_instance(s, inst)
    elif st == InstanceStatus.PROVISIONING:
        _check_provisioning(s, inst)
    elif st in (InstanceStatus.IDLE, InstanceStatus.BUSY):
        _check_instance(s, inst)
    elif st == InstanceStatus.TERMINATING:
        _terminate(s, inst)
    inst.last_processed_at = get_current_datetime()


# SSH-fleet deploys (upload agents, start the shim, wait for host_info: up to minutes per host) run
# on their own workers, never inside a reconciler claim: the pass that starts one returns at once,
# and the pass after the deploy finished applies its result.
_deploy_pool = None
_deploys: dict = {}


def _deploy_executor():
    global _deploy_pool
    if _deploy_pool is None:
        from concurrent.futures import ThreadPoolExecutor

        _deploy_pool = ThreadPoolExecutor(max_workers=8, thread_name_prefix="ssh-deploy")
    return _deploy_pool


# A deploy can take minutes (agent upload, shim start, host_info polling), so it is leased on the
# instance row: the replica that starts it records itself and the start time while it holds the
# row (claimed FOR UPDATE on Postgres), and every other replica skips the instance until the lease
# is older than the deploy deadline -- with several server replicas on one database a host is
# never deployed twice, and only the owner applies the result (reference: the instance lock held
# across the deploy, process_instances.py:210-377).
DEPLOY_LEASE = PROVISIONING_DEADLINE


def _add_remote(s: Session, inst: InstanceModel):
    from dstack_amd.server import settings

    me = settings.SERVER_REPLICA_ID
    now = get_current_datetime()
    fut = _deploys.get(inst.id)
    if fut is not None and not fut.done():
        return  # still deploying on its worker
    if fut is None:
        if inst.deploy_owner and inst.deploy_owner != me and inst.deploy_started_at and \
                now - inst.deploy_started_at < DEPLOY_LEASE:
            return  # another replica's deploy is in flight
        if now - inst.created_at > TERMINATION_DEADLINE_OFFSET:
            # never came up in time (unreachable host, bad key, broken agent): give up on it
            inst.status = InstanceStatus.TERMINATED.value
            inst.termination_reason = "Provisioning timeout expired"
            inst.deploy_owner = None
            return
        if inst.last_retry_at and now - inst.last_retry_at < SSH_DEPLOY_RETRY:
            return
        inst.last_retry_at = now
        inst.deploy_owner = me
        inst.deploy_started_at = now
        s.commit()  # the lease is visible to other replicas before the deploy starts
        rci = RemoteConnectionInfo.model_validate_json(inst.remote_connection_info)
        project = inst.project
        key = next((k.private for k in rci.ssh_keys if k.private), None) or project.ssh_private_key
        fut = _deploy_executor().submit(deploy_ssh_instance, rci, project.ssh_public_key, key)
        _deploys[inst.id] = fut
        fut.add_done_callback(lambda _f: scheduler.wake(scheduler.INSTANCES))
        if not fut.done():
            return
    _deploys.pop(inst.id, None)
    if inst.deploy_owner not in (None, me):
        return  # the lease expired and another replica took the host over: its deploy wins
    inst.deploy_owner = None
    inst.deploy_started_at = None
    rci = RemoteConnectionInfo.model_validate_json(inst.remote_connection_info)
    try:
        host_info = fut.result()
    except Exception as e:  # noqa: BLE001
        logger.warning("instance %s: SSH deploy failed: %s", inst.name, e)
        inst.termination_reason = f"deploy failed: {e}"[:4000]
        if get_current_datetime() - inst.created_at > TERMINATION_DEADLINE_OFFSET:
            inst.status = InstanceStatus.TERMINATED.value
        return
    itype, topo = host_info_to_instance_type(host_info)
    bd = json.loads(inst.backend_data or "{}")
    internal_ip = bd.get("internal_ip") or get_ip_from_network(bd.get("network"), host_info.get("addresses") or [])
    if internal_ip is None and bd.get("network"):
        inst.termination_reason = f"no address in network {bd.get('network')}"
        inst.status = InstanceStatus.TERMINATED.value
        return
    try:
        total_blocks = split_blocks(topo, bd.get("blocks", 1), itype.resources.cpus)
    except ProvisioningError as e:
        inst.termination_reason = str(e)
        inst.status = InstanceStatus.TERMINATED.value
        return
    jpd = JobProvisioningData(
        backend=BackendType.REMOTE, instance_type=itype, instance_id=inst.name, hostname=rci.host,
        internal_ip=internal_ip or rci.host, region="remote", price=0.0, username=rci.ssh_user, ssh_port=rci.port,
        dockerized=True, backend_data=remote_backend_data(direct=bool(bd.get("direct"))),
    )
    offer = InstanceOfferWithAvailability(backend=BackendType.REMOTE, instance=itype, region="remote", price=0.0,
                                          availability=InstanceAvailability.AVAILABLE, total_blocks=total_blocks)
    inst.job_provisioning_data = jpd.model_dump_json()
    inst.offer = offer.model_dump_json()
    inst.host_topology = topo.model_dump_json()
    inst.total_blocks = total_blocks
    inst.status = InstanceStatus.IDLE.value
    inst.started_at = get_current_datetime()
    inst.termination_reason = None
    scheduler.wake(scheduler.SUBMITTED_JOBS)


NO_CAPACITY_RETRY = timedelta(minutes=1)
# GPU health: the shim probes at start; the server re-reads it at most once a minute per instance
# and asks for a fresh probe when the last one is older than this (only while the host is idle)
GPU_PROBE_MAX_AGE = timedelta(hours=6)
GPU_HEALTH_POLL = 60.0
_health_polled: dict = {}
MAX_OFFERS_TRIED = 15


def _create_instance(s: Session, inst: InstanceModel):
    """Provision a cloud-fleet instance (reference ``_create_instance``, process_instances.py:431-605).

    * ``placement: cluster`` fleets: instances after the first wait until it is provisioned, then
      take offers only from its backend and region (same availability zone, and an AWS placement
      group created once per fleet/backend/region), so the nodes share a network fabric;
    * no offers / every offer failed: with ``retry.on_events: [no-capacity]`` try again every
      minute until the retry duration expires, otherwise the instance is terminated;
    * ``blocks`` of the fleet split the new instance's GPUs for shared use."""
    now = get_current_datetime()
    if inst.last_retry_at is not None and now - inst.last_retry_at < NO_CAPACITY_RETRY:
        return
    project = inst.project
    profile = Profile.model_validate_json(inst.profile) if inst.profile else Profile(name="default")
    req = Requirements.model_validate_json(inst.requirements) if inst.requirements else None
    if req is None:
        inst.status = InstanceStatus.TERMINATED.value
        inst.termination_reason = "no requirements"
        return
    bd = json.loads(inst.backend_data or "{}")
    cluster = bd.get("placement") == InstanceGroupPlacement.CLUSTER.value
    master_jpd: Optional[JobProvisioningData] = None
    if cluster and inst.fleet is not None:
        master = min(inst.fleet.instances, key=lambda i: (i.instance_num, i.created_at))
        if master.id != inst.id:
            if master.job_provisioning_data is None:
                if master.status != InstanceStatus.TERMINATED.value:
                    return  # wait for the first node: the others follow it
            else:
                master_jpd = JobProvisioningData.model_validate_json(master.job_provisioning_data)
    from dstack_amd.server.services.jobs.configurators import retry_from_profile

    retry = retry_from_profile(profile)
    should_retry = retry is not None and RetryEvent.NO_CAPACITY in retry.on_events
    if retry is not None and now > inst.created_at + timedelta(seconds=retry.duration):
        inst.status = InstanceStatus.TERMINATED.value
        inst.termination_reason = "Retry duration expired"
        return
    blocks = bd.get("blocks", 1) or 1
    offers = offers_services.get_offers_by_requirements(
        s, project, profile, req, exclude_not_available=True, multinode=cluster,
        master_job_provisioning_data=master_jpd, blocks=blocks)
    offers = [(c, o) for c, o in offers
              if o.backend in BACKENDS_WITH_CREATE_INSTANCE_SUPPORT and o.backend != BackendType.REMOTE]
    cfg = InstanceConfiguration(project_name=project.name, instance_name=inst.name, user="",
                                ssh_keys=[SSHKey(public=project.ssh_public_key.strip())],
                                availability_zone=master_jpd.availability_zone if master_jpd else None,
                                reservation=profile.reservation)
    for compute, offer in offers[:MAX_OFFERS_TRIED]:
        if cluster and inst.fleet is not None and offer.backend in BACKENDS_WITH_PLACEMENT_GROUPS_SUPPORT:
            try:
                cfg.placement_group_name = _fleet_placement_group(s, inst, compute, offer)
            except Exception as e:  # noqa: BLE001
                logger.info("instance %s: placement group in %s/%s failed: %s", inst.name, offer.backend.value,
                            offer.region, e)
                continue
        try:
            jpd = compute.create_instance(offer, cfg)
        except Exception as e:  # noqa: BLE001
            logger.info("instance %s: %s/%s failed: %s", inst.name, offer.backend.value, offer.instance.name, e)
            continue
        inst.backend = jpd.backend.value
        inst.region = jpd.region
        inst.price = jpd.price
        inst.offer = offer.model_dump_json()
        inst.job_provisioning_data = jpd.model_dump_json()
        res = offer.instance.resources
        inst.total_blocks = auto_blocks(len(res.gpus), res.cpus) if blocks == "auto" else int(blocks)
        inst.backend_data = jpd.backend_data
        inst.status = (InstanceStatus.IDLE if jpd.backend == BackendType.LOCAL else InstanceStatus.PROVISIONING).value
        inst.started_at = now
        inst.termination_reason = None
        if jpd.backend == BackendType.LOCAL:
            from dstack_amd.core.backends.local import LocalShim

            _, topo = host_info_to_instance_type(LocalShim.get().host_info)
            inst.host_topology = topo.model_dump_json()
        return
    inst.last_retry_at = now
    inst.termination_reason = "no offers / no capacity" if not offers else "all offers failed"
    if not should_retry:
        inst.status = InstanceStatus.TERMINATED.value


def _fleet_placement_group(s: Session, inst: InstanceModel, compute, offer) -> str:
    """The fleet's cluster placement group in the offer's backend/region (created on first use)."""
    from dstack_amd.core.models.placement import PlacementGroup, PlacementGroupConfiguration
    from dstack_amd.server.models import PlacementGroupModel

    for pg in s.execute(select(PlacementGroupModel).where(PlacementGroupModel.fleet_id == inst.fleet_id,
                                                          PlacementGroupModel.deleted == False)).scalars():  # noqa
        c = PlacementGroupConfiguration.model_validate_json(pg.configuration)
        if c.backend == offer.backend and c.region == offer.region:
            return pg.name
    conf = PlacementGroupConfiguration(backend=offer.backend, region=offer.region)
    name = f"{inst.project.name}-{inst.fleet.name}-{uuid.uuid4().hex[:8]}-pg"
    pgpd = compute.create_placement_group(PlacementGroup(name=name, project_name=inst.project.name,
                                                         configuration=conf))
    s.add(PlacementGroupModel(id=uuid.uuid4(), name=name, project_id=inst.project_id, fleet_id=inst.fleet_id,
                              configuration=conf.model_dump_json(), provisioning_data=pgpd.model_dump_json()))
    s.flush()
    return name


def _check_provisioning(s: Session, inst: InstanceModel):
    jpd = pools_services.instance_jpd(inst)
    if jpd is None:
        return
    if not jpd.hostname:
        try:
            compute = backends_services.get_project_backend(s, inst.project, jpd.backend)
            compute.update_provisioning_data(jpd, inst.project.ssh_public_key, inst.project.ssh_private_key)
            inst.job_provisioning_data = jpd.model_dump_json()
        except Exception as e:  # noqa: BLE001
            logger.debug("update_provisioning_data: %s", e)
    if jpd.hostname and _shim_healthy(inst, jpd):
        driver_err = _gpu_driver_error(inst, jpd)
        if driver_err:
            # the bootstrap could not load amdgpu (no /dev/kfd): a GPU host without GPUs is a
            # failed provisioning, with the bootstrap's reason, not an idle CPU host
            inst.status = InstanceStatus.TERMINATING.value
            inst.termination_reason = f"GPU driver: {driver_err}"[:1000]
            inst.health_status = inst.termination_reason
            inst.termination_deadline = inst.termination_deadline or get_current_datetime()
            logger.warning("%s: %s", inst.name, inst.termination_reason)
            return
        inst.status = (InstanceStatus.BUSY if (inst.busy_blocks or 0) > 0 else InstanceStatus.IDLE).value
        inst.termination_deadline = None
        inst.health_status = None
        inst.unreachable = False
        refresh_gpu_health(inst, jpd, force=True)
        scheduler.wake(scheduler.RUNNING_JOBS, scheduler.SUBMITTED_JOBS)
        return
    now = get_current_datetime()
    inst.health_status = "waiting for the cloud to report the host" if not jpd.hostname else "shim not reachable yet"
    if now - (inst.started_at or inst.created_at) > PROVISIONING_DEADLINE:
        inst.status = InstanceStatus.TERMINATING.value
        inst.termination_reason = "provisioning timeout"
        inst.termination_deadline = inst.termination_deadline or now


def refresh_gpu_health(inst: InstanceModel, jpd: JobProvisioningData, force: bool = False) -> Optional[str]:
    """Copy the shim's asynchronous HIP probe result (HBM TB/s, MFMA TFLOPS vs 80 % of the per-SKU
    baseline) into the instance's health; an unhealthy host is skipped by the scheduler
    (``pools.filter_pool_instances``).  A stale result is refreshed by asking the shim for a new
    probe while the host runs no job.  Never on a job's critical path.  Returns the shim state."""
    import time as _time

    from dstack_amd.core.models.instances import InstanceHealth

    now = _time.monotonic()
    if not force and now - _health_polled.get(inst.id, -1e9) < GPU_HEALTH_POLL:
        return None
    _health_polled[inst.id] = now
    try:
        shim = get_shim_client(jpd, inst.project.ssh_private_key)
        doc = shim.gpu_health()
    except Exception as e:  # noqa: BLE001 - health is advisory; reachability is judged elsewhere
        logger.debug("%s: gpu health unavailable: %s", inst.name, e)
        return None
    if not isinstance(doc, dict):
        return None  # a shim without the endpoint
    state = doc.get("state")
    res = doc.get("result") or None
    ran_at = (doc.get("ran_at_ms") or 0) / 1000.0
    old = json.loads(inst.health_data) if inst.health_data else {}
    if res and state in ("done", "failed") and ran_at and ran_at != old.get("ran_at"):
        try:
            h = InstanceHealth(healthy=bool(res.get("healthy", False)), hbm_tb_s=res.get("hbm_tb_s"),
                               mfma_bf16_tflops=res.get("mfma_bf16_tflops"), mfma_fp8_tflops=res.get("mfma_fp8_tflops"),
                               xgmi_gb_s=res.get("xgmi_gb_s"), rccl_busbw_gb_s=res.get("rccl_busbw_gb_s"),
                               message=res.get("message") or ("" if res.get("healthy") else "GPU health probe failed"),
                               sku=res.get("sku"), thresholds=res.get("thresholds"), ran_at=ran_at, source="shim")
        except Exception:  # noqa: BLE001 - a malformed document must not break the pass
            return state
        inst.health_data = h.model_dump_json()
        inst.health_status = None  # (only called with the shim reachable)
        if not h.healthy:
            inst.health_status = f"GPU health probe: {h.message}"
            logger.warning("%s: GPU health probe failed: %s", inst.name, h.message)
        old = json.loads(inst.health_data)
    stale = not old.get("ran_at") or _time.time() - old["ran_at"] > GPU_PROBE_MAX_AGE.total_seconds()
    if stale and state in ("idle", "done", "failed", "interrupted") and (inst.busy_blocks or 0) == 0 and \
            inst.status == InstanceStatus.IDLE.value:
        try:
            state = shim.start_gpu_probe()
        except Exception as e:  # noqa: BLE001
            logger.debug("%s: start probe: %s", inst.name, e)
    return state


def _gpu_driver_error(inst: InstanceModel, jpd: JobProvisioningData) -> Optional[str]:
    """The shim's ``gpu_driver_error`` (bootstrap marker) when the offer has GPUs but the host
    reports none; None otherwise or when host_info is unavailable."""
    if not jpd.instance_type.resources.gpus:
        return None
    try:
        hi = get_shim_client(jpd, inst.project.ssh_private_key).host_info()
    except Exception:  # noqa: BLE001 - older shims / transient errors: judged by the probes later
        return None
    if not isinstance(hi, dict) or int(hi.get("gpu_count") or 0) > 0:
        return None
    return hi.get("gpu_driver_error") or None


def _shim_healthy(inst: InstanceModel, jpd: JobProvisioningData) -> bool:
    try:
        return get_shim_client(jpd, inst.project.ssh_private_key).healthcheck() is not None
    except Exception:  # noqa: BLE001
        return False


def _check_instance(s: Session, inst: InstanceModel):
    jpd = pools_services.instance_jpd(inst)
    if jpd is None:
        return
    now = get_current_datetime()
    healthy = _shim_healthy(inst, jpd) if jpd.dockerized else True
    if healthy:
        inst.unreachable = False
        inst.termination_deadline = None
        gpu = json.loads(inst.health_data) if inst.health_data else {}
        inst.health_status = None if gpu.get("healthy", True) else f"GPU health probe: {gpu.get('message', '')}"
        if jpd.dockerized:
            refresh_gpu_health(inst, jpd)
    else:
        inst.unreachable = True
        inst.health_status = "shim unreachable"
        if inst.termination_deadline is None:
            inst.termination_deadline = now + TERMINATION_DEADLINE_OFFSET
        elif now > inst.termination_deadline and jpd.backend != BackendType.REMOTE:
            inst.status = InstanceStatus.TERMINATING.value
            inst.termination_reason = "unreachable"
            return
    if inst.status == InstanceStatus.IDLE.value and (inst.busy_blocks or 0) == 0:
        idle_limit = inst.termination_idle_time
        if idle_limit is not None and idle_limit >= 0 and inst.termination_policy != "dont-destroy":
            since = inst.last_job_processed_at or inst.started_at or inst.created_at
            if now - since > timedelta(seconds=idle_limit):
                inst.status = InstanceStatus.TERMINATING.value
                inst.termination_reason = "idle timeout"
                scheduler.wake(scheduler.INSTANCES)


TERMINATION_RETRY_INTERVAL = timedelta(minutes=1)
TERMINATION_RETRY_MAX = timedelta(minutes=15)


def _terminate(s: Session, inst: InstanceModel):
    """Terminate the cloud instance; a failed call is retried at most once a minute and given up
    (the instance is marked terminated) 15 minutes after the first failure (reference
    process_instances ``_terminate``)."""
    jpd = pools_services.instance_jpd(inst)
    if inst.last_termination_retry_at is not None and \
            get_current_datetime() - inst.last_termination_retry_at < TERMINATION_RETRY_INTERVAL:
        return  # too early to retry
    if jpd is not None and jpd.backend not in (BackendType.REMOTE, BackendType.LOCAL):
        try:
            compute = backends_services.get_project_backend(s, inst.project, jpd.backend)
            compute.terminate_instance(jpd.instance_id, jpd.region, jpd.backend_data)
        except Exception as e:  # noqa: BLE001
            now = get_current_datetime()
            inst.first_termination_retry_at = inst.first_termination_retry_at or now
            inst.last_termination_retry_at = now
            if now - inst.first_termination_retry_at < TERMINATION_RETRY_MAX:
                logger.warning("instance %s: terminate failed (will retry): %s", inst.name, e)
                return
    inst.status = InstanceStatus.TERMINATED.value
    inst.finished_at = get_current_datetime()
    inst.deleted = True
    inst.deleted_at = get_current_datetime()
    scheduler.wake(scheduler.FLEETS)


