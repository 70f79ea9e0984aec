"""SUBMITTED -> PROVISIONING (reference: ``S/background/tasks/process_submitted_jobs.py:83-707``).

1. multinode gating: workers wait for the master job's provisioning data (same backend/region);
2. reuse a pool instance (cheapest idle first; shared instances by GPU blocks) — GPUs inside the
   instance are chosen xGMI-topology-aware (``services/topology.py``);
3. otherwise provision on a new instance through the backends (<= 15 offers), creating an
   instance model and, for a run without one, an autocreated fleet (``placement: cluster`` for
   multinode).
"""

from __future__ import annotations

import json
import logging
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import BackendError, ComputeError, NoCapacityError, ServerClientError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models import images
from dstack_amd.core.models.common import NetworkMode
from dstack_amd.core.models.instances import InstanceOfferWithAvailability, InstanceStatus
from dstack_amd.core.models.profiles import DEFAULT_RUN_TERMINATION_IDLE_TIME, CreationPolicy
from dstack_amd.core.models.runs import (
    Job,
    JobProvisioningData,
    JobRuntimeData,
    JobStatus,
    JobTerminationReason,
    RunSpec,
    RunStatus,
)
from dstack_amd.server import settings
from dstack_amd.server.background import scheduler
from dstack_amd.server.background.common import claim_and_process
from dstack_amd.server.models import FleetModel, InstanceModel, JobModel, RunModel
from dstack_amd.server.services import fleets as fleets_services
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.server.services import offers as offers_services
from dstack_amd.server.services import pools as pools_services
from dstack_amd.server.services import runs as runs_services
from dstack_amd.server.services.jobs import volumes as job_volumes
from dstack_amd.server.services.locking import lockset, release_at_transaction_end
from dstack_amd.server.services.topology import busy_set, pick_gpus
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)


def process_submitted_jobs(batch: int = 5) -> bool:
    def select_ids(s: Session):
        return s.execute(select(JobModel.id).where(JobModel.status == JobStatus.SUBMITTED.value)
                         .order_by(JobModel.last_processed_at).limit(batch * 4)).scalars()

    return claim_and_process("jobs", select_ids, _process_job, batch)


def _process_job(s: Session, job_id):
    job = s.get(JobModel, job_id)
    if job is None or job.status != JobStatus.SUBMITTED.value:
        return
    run: RunModel = job.run
    if RunStatus(run.status) in (RunStatus.TERMINATING,) or RunStatus(run.status).is_finished():
        return
    run_spec = RunSpec.model_validate_json(run.run_spec)
    spec = jobs_services.job_spec(job)
    profile = run_spec.merged_profile
    multinode = spec.jobs_per_replica > 1
    master_jpd: Optional[JobProvisioningData] = None
    if spec.job_num != 0:
        master = _master_job(run, job)
        if master is None or master.job_provisioning_data is None:
            job.last_processed_at = get_current_datetime()
            return  # wait for the master job to be provisioned
        master_jpd = jobs_services.job_jpd(master)
    fleet = s.get(FleetModel, run.fleet_id) if run.fleet_id else None
    # network volumes pin the job to their backend/region (attached in process_running_jobs)
    try:
        volumes = job_volumes.get_job_configured_volumes(s, run.project, spec)
        job_volumes.check_can_attach_job_volumes(volumes)
    except ServerClientError as e:
        jobs_services.terminate_job(job, JobTerminationReason.VOLUME_ERROR, str(e), delay=False)
        scheduler.wake(scheduler.TERMINATING_JOBS, scheduler.RUNS)
        return
    # ---- 1) reuse a pool instance ----
    if _assign_pool_instance(s, run, job, spec, profile, fleet, multinode, master_jpd, volumes):
        scheduler.wake(scheduler.RUNNING_JOBS, scheduler.RUNS)
        return
    if profile.creation_policy == CreationPolicy.REUSE:
        _no_capacity(job, "No idle instance matches the requirements (creation_policy: reuse)")
        return
    if fleet is not None and not _fleet_can_grow(fleet):
        _no_capacity(job, f"No idle instance in fleet {fleet.name} matches the requirements")
        return
    # ---- 2) provision a new instance ----
    offers = offers_services.get_offers_by_requirements(
        s, run.project, profile, spec.requirements, exclude_not_available=True, multinode=multinode,
        master_job_provisioning_data=master_jpd, privileged=spec.privileged,
        instance_mounts=_has_required_instance_mounts(spec),
    )
    offers = [(c, o) for c, o in offers if o.backend != BackendType.REMOTE]
    offers = job_volumes.filter_offers_by_volumes(offers, volumes)
    n_before = len(offers)
    offers = [(c, o) for c, o in offers if images.offer_supported(spec.image_name, o.instance.resources.gpus)]
    if not offers:
        _no_capacity(job, "No offers match the requirements" if not n_before else
                     f"No offers match the requirements: image {spec.image_name} names a ROCm too old for "
                     f"the offered GPUs (MI350X/MI355X need ROCm >= 7.0)")
        return
    run_model = runs_services.run_model_to_run(run, include_jobs=False)
    job_obj = Job(job_spec=spec, job_submissions=[jobs_services.job_model_to_job_submission(job)])
    for compute, offer in offers[: settings.MAX_OFFERS_TRIED]:
        try:
            jpd = compute.run_job(run_model, job_obj, offer, run.project.ssh_public_key, run.project.ssh_private_key,
                                  [])
        except (NoCapacityError, BackendError, ComputeError, NotImplementedError) as e:
            logger.info("%s: offer %s/%s failed: %s", job.job_name, offer.backend.value, offer.instance.name, e)
            continue
        _create_instance_for_job(s, run, job, spec, offer, jpd, profile, fleet, multinode)
        scheduler.wake(scheduler.RUNNING_JOBS, scheduler.RUNS, scheduler.INSTANCES)
        return
    _no_capacity(job, "All offers failed")


def _master_job(run: RunModel, job: JobModel) -> Optional[JobModel]:
    cands = [j for j in run.jobs if j.replica_num == job.replica_num and j.job_num == 0]
    return max(cands, key=lambda j: j.submission_num) if cands else None


def _has_required_instance_mounts(spec) -> bool:
    return jobs_services.has_required_instance_mounts(spec)


def _fleet_can_grow(fleet: FleetModel) -> bool:
    """A run bound to a fleet gets a new instance in it when the fleet is autocreated, or a cloud
    fleet below its ``nodes.max`` (SSH fleets have exactly their hosts)."""
    try:
        spec = json.loads(fleet.spec)
    except ValueError:
        return False
    if spec.get("autocreated"):
        return True
    conf = spec.get("configuration") or {}
    if conf.get("ssh_config"):
        return False
    nodes = conf.get("nodes") or {}
    nmax = nodes.get("max") if isinstance(nodes, dict) else nodes
    active = [i for i in fleet.instances if not i.deleted and i.status != InstanceStatus.TERMINATED.value]
    return nmax is None or len(active) < int(nmax)


def _no_capacity(job: JobModel, msg: str):
    jobs_services.terminate_job(job, JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY, msg, delay=False)
    scheduler.wake(scheduler.TERMINATING_JOBS, scheduler.RUNS)


def _runtime_data(inst_offer: InstanceOfferWithAvailability, gpu_indices: Optional[List[int]], spec) -> JobRuntimeData:
    res = inst_offer.instance.resources
    shared = inst_offer.total_blocks > 1
    bridge = shared or settings.FORCE_BRIDGE_NETWORK  # DSTACK_FORCE_BRIDGE_NETWORK
    return JobRuntimeData(
        network_mode=NetworkMode.BRIDGE if bridge else NetworkMode.HOST,
        gpu=len(res.gpus) if shared else None, cpu=float(res.cpus) if shared else None,
        memory=(res.memory_mib / 1024) if shared else None, offer=inst_offer, gpu_indices=gpu_indices,
    )


def _gpu_request(spec, offer: InstanceOfferWithAvailability) -> int:
    g = spec.requirements.resources.gpu
    if g is None or (g.count.max == 0):
        return 0
    return len(offer.instance.resources.gpus)


def _assign_pool_instance(s: Session, run: RunModel, job: JobModel, spec, profile, fleet, multinode: bool,
                          master_jpd, volumes=()) -> bool:
    instances = pools_services.list_project_instances(s, run.project)
    cands = pools_services.filter_pool_instances(instances, profile, spec.requirements, fleet=fleet,
                                                 multinode=multinode, master_jpd=master_jpd)
    cands = [(i, sh) for i, sh in cands if job_volumes.instance_matches_volumes(i, volumes)
             and images.offer_supported(spec.image_name, sh.instance.resources.gpus)]
    if not cands:
        return False
    ls = lockset("instances")
    for inst, shared in cands:
        if not ls.try_add_many([inst.id]):
            continue
        assigned = False
        try:
            s.refresh(inst)
            shared = pools_services.get_instance_shared_offer(inst, spec.requirements)
            if shared is None:
                continue
            n_gpus = _gpu_request(spec, shared)
            topo = pools_services.instance_topology(inst)
            gpu_indices = None
            if n_gpus and topo is not None and topo.gpus and inst.backend != BackendType.LOCAL.value:
                busy = busy_set(inst.busy_gpus)
                free = [g.index for g in topo.gpus if g.index not in busy]
                gpu_indices = pick_gpus(topo, free, n_gpus)
                if gpu_indices is None:
                    continue
                inst.busy_gpus = ",".join(str(x) for x in sorted(busy + gpu_indices))
            inst.busy_blocks = (inst.busy_blocks or 0) + shared.blocks
            inst.status = InstanceStatus.BUSY.value
            job.instance_id = inst.id
            job.instance_assigned = True
            job.job_provisioning_data = inst.job_provisioning_data
            job.job_runtime_data = _runtime_data(shared, gpu_indices, spec).model_dump_json()
            job.status = JobStatus.PROVISIONING.value
            job.last_processed_at = get_current_datetime()
            jobs_services.mark_timing(job, "assigned")
            if run.fleet_id is None:
                run.fleet_id = inst.fleet_id
            s.flush()
            assigned = True
            return True
        finally:
            if assigned:  # BUSY must be committed before another thread may re-read the instance
                release_at_transaction_end(s, ls, [inst.id])
            else:
                ls.remove_many([inst.id])
    return False


def _create_instance_for_job(s: Session, run: RunModel, job: JobModel, spec, offer, jpd: JobProvisioningData, profile,
                             fleet: Optional[FleetModel], multinode: bool):
    project = run.project
    if fleet is None:
        fleet = fleets_services.create_autocreated_fleet(s, project, run.run_name, profile, multinode)
        run.fleet_id = fleet.id
    pool = pools_services.get_or_create_default_pool(s, project)
    idle = profile.idle_duration
    idle_s = DEFAULT_RUN_TERMINATION_IDLE_TIME if idle is None else int(idle)
    ready = jpd.backend == BackendType.LOCAL  # the local shim is already up
    inst = pools_services.create_instance_model(
        s, project, pool, name=f"{run.run_name}-{spec.job_num}-{spec.replica_num}",
        status=InstanceStatus.BUSY if ready else InstanceStatus.PROVISIONING, fleet=fleet,
        instance_num=len(fleet.instances), backend=jpd.backend.value, region=jpd.region, price=jpd.price,
        job_provisioning_data=jpd.model_dump_json(), offer=offer.model_dump_json(), total_blocks=1, busy_blocks=1,
        profile=profile.model_dump_json(), requirements=spec.requirements.model_dump_json(),
        termination_idle_time=idle_s, termination_policy="destroy-after-idle" if idle_s >= 0 else "dont-destroy",
        backend_data=jpd.backend_data,
    )
    if jpd.backend == BackendType.LOCAL:
        from dstack_amd.core.backends.local import LocalShim
        from dstack_amd.core.backends.remote import host_info_to_instance_type

        _, topo = host_info_to_instance_type(LocalShim.get().host_info)
        inst.host_topology = topo.model_dump_json()
    gpu_indices = None
    n_gpus = _gpu_request(spec, offer)
    topo = pools_services.instance_topology(inst)
    # local backend: every local instance is the same host behind ONE shim, whose xGMI-aware lock
    # arbitrates between them; pinning indices per instance row would hand two jobs the same GPUs
    if n_gpus and topo is not None and topo.gpus and jpd.backend != BackendType.LOCAL:
        gpu_indices = pick_gpus(topo, [g.index for g in topo.gpus], n_gpus)
        inst.busy_gpus = ",".join(str(x) for x in (gpu_indices or []))
    job.instance_id = inst.id
    job.instance_assigned = True
    job.job_provisioning_data = jpd.model_dump_json()
    job.job_runtime_data = _runtime_data(offer, gpu_indices, spec).model_dump_json()
    job.status = JobStatus.PROVISIONING.value
    job.last_processed_at = get_current_datetime()
    jobs_services.mark_timing(job, "provisioned")
    s.flush()
