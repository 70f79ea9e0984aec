"""Jobs service: model conversion, termination and instance release (reference:
``S/services/jobs/__init__.py:65-611``)."""

from __future__ import annotations

import json
import logging
import uuid
from datetime import timedelta
from typing import Dict, List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import SSHError
from dstack_amd.core.models.instances import InstanceStatus
from dstack_amd.core.models.runs import (
    Job,
    JobProvisioningData,
    JobRuntimeData,
    JobSpec,
    JobStatus,
    JobSubmission,
    JobTerminationReason,
    RunSpec,
)
from dstack_amd.server.models import InstanceModel, JobModel, ProjectModel, RunModel
from dstack_amd.server.services.jobs.configurators import get_job_specs_from_run_spec
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)

REMOVE_DELAY = timedelta(seconds=15)  # give the runner time to flush logs after stop


def get_jobs_from_run_spec(run_spec: RunSpec, replica_num: int, secrets: Optional[Dict[str, str]] = None):
    return get_job_specs_from_run_spec(run_spec, replica_num, secrets)


def job_spec(job: JobModel) -> JobSpec:
    return JobSpec.model_validate_json(job.job_spec_data)


def job_jpd(job: JobModel) -> Optional[JobProvisioningData]:
    return JobProvisioningData.model_validate_json(job.job_provisioning_data) if job.job_provisioning_data else None


def job_jrd(job: JobModel) -> Optional[JobRuntimeData]:
    return JobRuntimeData.model_validate_json(job.job_runtime_data) if job.job_runtime_data else None


def job_timings(job: JobModel) -> Dict[str, float]:
    return json.loads(job.timings) if job.timings else {}


def mark_timing(job: JobModel, stage: str, ts: Optional[float] = None):
    t = job_timings(job)
    if stage not in t:
        t[stage] = ts if ts is not None else get_current_datetime().timestamp()
        job.timings = json.dumps(t)


def job_model_to_job_submission(job: JobModel) -> JobSubmission:
    return JobSubmission(
        id=job.id, submission_num=job.submission_num, submitted_at=job.submitted_at,
        last_processed_at=job.last_processed_at, finished_at=job.finished_at, status=JobStatus(job.status),
        termination_reason=JobTerminationReason(job.termination_reason) if job.termination_reason else None,
        termination_reason_message=job.termination_reason_message, exit_status=job.exit_status,
        job_provisioning_data=job_jpd(job), job_runtime_data=job_jrd(job), timings=job_timings(job) or None,
    )


def group_jobs_by_replica_latest(jobs: List[JobModel]) -> Dict[int, List[JobModel]]:
    """replica_num -> latest submission of each job_num (``group_jobs_by_replica_latest``)."""
    latest: Dict[tuple, JobModel] = {}
    for j in jobs:
        key = (j.replica_num, j.job_num)
        if key not in latest or j.submission_num > latest[key].submission_num:
            latest[key] = j
    out: Dict[int, List[JobModel]] = {}
    for (r, _), j in sorted(latest.items()):
        out.setdefault(r, []).append(j)
    return out


def terminate_job(job: JobModel, reason: JobTerminationReason, message: Optional[str] = None, delay: bool = True):
    """Move a job to TERMINATING; the runner is asked to stop first (graceful) and the container
    is removed by ``process_terminating_jobs`` after ``remove_at``."""
    if JobStatus(job.status).is_finished() or job.status == JobStatus.TERMINATING.value:
        return
    job.status = JobStatus.TERMINATING.value
    job.termination_reason = reason.value
    if message:
        job.termination_reason_message = message
    job.remove_at = get_current_datetime() + (REMOVE_DELAY if delay else timedelta(0))
    job.last_processed_at = get_current_datetime()


def stop_runner(s: Session, job: JobModel):
    """Best-effort graceful stop (SIGINT via the runner's /api/stop)."""
    jpd = job_jpd(job)
    if jpd is None or job.status not in (JobStatus.RUNNING.value, JobStatus.TERMINATING.value):
        return
    from dstack_amd.server.services.runner.client import get_runner_client

    project = s.get(ProjectModel, job.project_id)
    try:
        get_runner_client(jpd, job_jrd(job), project.ssh_private_key).stop()
    except (SSHError, Exception) as e:  # noqa: BLE001
        logger.debug("stop_runner %s: %s", job.job_name, e)


def release_instance(s: Session, job: JobModel):
    """Free the job's blocks/GPUs on its instance (``process_terminating_job`` tail)."""
    if job.instance_id is None:
        return
    inst = s.get(InstanceModel, job.instance_id)
    job.used_instance_id = job.instance_id
    job.instance_id = None
    if inst is None:
        return
    jrd = job_jrd(job)
    blocks = jrd.offer.blocks if jrd and jrd.offer else (inst.total_blocks or 1)
    inst.busy_blocks = max(0, (inst.busy_blocks or 0) - blocks)
    if jrd and jrd.gpu_indices:
        busy = {int(x) for x in inst.busy_gpus.split(",") if x != ""}
        busy -= set(jrd.gpu_indices)
        inst.busy_gpus = ",".join(str(x) for x in sorted(busy))
    if inst.status == InstanceStatus.BUSY.value and inst.busy_blocks == 0:
        inst.status = InstanceStatus.IDLE.value
    inst.last_job_processed_at = get_current_datetime()


def get_job_secrets(s: Session, project: ProjectModel) -> Dict[str, str]:
    from dstack_amd.server.services.secrets import get_project_secrets_mapping

    return get_project_secrets_mapping(s, project)


def list_run_jobs(s: Session, run: RunModel) -> List[JobModel]:
    return list(s.execute(select(JobModel).where(JobModel.run_id == run.id)
                          .order_by(JobModel.replica_num, JobModel.job_num, JobModel.submission_num)).scalars())


def new_job_model(run: RunModel, spec: JobSpec, submission_num: int = 0) -> JobModel:
    now = get_current_datetime()
    j = JobModel(
        id=uuid.uuid4(), project_id=run.project_id, run_id=run.id, run_name=run.run_name, job_num=spec.job_num,
        job_name=spec.job_name, replica_num=spec.replica_num, submission_num=submission_num, submitted_at=now,
        last_processed_at=now, status=JobStatus.SUBMITTED.value, job_spec_data=spec.model_dump_json(),
    )
    j.timings = json.dumps({"submitted": now.timestamp()})
    return j


def has_required_instance_mounts(spec) -> bool:
    """Non-optional instance mounts need a VM backend (a host path to bind); optional ones do not
    restrict the offers (reference: ``check_run_spec_has_instance_mounts``)."""
    from dstack_amd.core.models.volumes import InstanceMountPoint

    return any(isinstance(mp, InstanceMountPoint) and not mp.optional for mp in spec.mount_points())
