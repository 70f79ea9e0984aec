"""TERMINATING -> final status (reference: ``S/background/tasks/process_terminating_jobs.py:22-93``,
``S/services/jobs/__init__.py:212-334``): stop + remove the container through the shim, detach
volumes, release the instance's blocks/GPUs."""

from __future__ import annotations

import logging
from datetime import timedelta

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.models.configurations import ServiceConfiguration
from dstack_amd.core.models.runs import JobStatus, JobTerminationReason, RunSpec
from dstack_amd.server.background import scheduler
from dstack_amd.server.background.common import claim_and_process
from dstack_amd.server.models import JobModel
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.server.services.runner.client import get_runner_client, get_shim_client
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)


def process_terminating_jobs(batch: int = 5) -> bool:
    def select_ids(s: Session):
        now = get_current_datetime()
        return s.execute(select(JobModel.id).where(JobModel.status == JobStatus.TERMINATING.value)
                         .where((JobModel.remove_at == None) | (JobModel.remove_at <= now))  # noqa: E711
                         .order_by(JobModel.last_processed_at).limit(batch * 4)).scalars()

    more = claim_and_process("jobs", select_ids, _process_job, batch)
    return more


def _detach_volumes(s: Session, job: JobModel) -> bool:
    from dstack_amd.server.services.jobs.volumes import detach_job_volumes

    try:
        return detach_job_volumes(s, job, job.used_instance_id, job.volumes_detached_at)
    except Exception as e:  # noqa: BLE001 - a broken backend must not wedge termination forever
        logger.warning("%s: volume detach failed: %s", job.job_name, e)
        return get_current_datetime() - job.volumes_detached_at > timedelta(minutes=10)


def _process_job(s: Session, job_id):
    job = s.get(JobModel, job_id)
    if job is None or job.status != JobStatus.TERMINATING.value:
        return
    if job.remove_at is not None and job.remove_at > get_current_datetime():
        return
    run = job.run
    jpd = jobs_services.job_jpd(job)
    reason = JobTerminationReason(job.termination_reason) if job.termination_reason else \
        JobTerminationReason.TERMINATED_BY_SERVER
    if jpd is not None and job.instance_id is not None:
        key = run.project.ssh_private_key
        if jpd.dockerized:
            try:
                shim = get_shim_client(jpd, key)
                spec = jobs_services.job_spec(job)
                shim.terminate_task(str(job.id), reason.value, job.termination_reason_message or "",
                                    timeout=min(int(spec.stop_duration or 10), 30))
                shim.remove_task(str(job.id))
            except Exception as e:  # noqa: BLE001
                logger.info("%s: shim terminate failed: %s", job.job_name, e)
        else:
            try:
                get_runner_client(jpd, jobs_services.job_jrd(job), key).stop()
            except Exception:  # noqa: BLE001
                pass
    if isinstance(RunSpec.model_validate_json(run.run_spec).configuration, ServiceConfiguration):
        from dstack_amd.server.services.services import unregister_replica

        unregister_replica(s, run, job)
    if job.volumes_detached_at is None:
        # the container is gone: the instance's blocks are freed right away, so a volume stuck in
        # detaching never holds the host (or its termination); detaching goes on against the
        # instance the job ran on (``used_instance_id``) -- soft first, forced after stop_duration
        job.volumes_detached_at = get_current_datetime()
        jobs_services.release_instance(s, job)
    if not _detach_volumes(s, job):
        job.last_processed_at = get_current_datetime()
        return  # retried on the next pass
    job.status = reason.to_status().value
    job.finished_at = get_current_datetime()
    job.last_processed_at = get_current_datetime()
    scheduler.wake(scheduler.RUNS, scheduler.SUBMITTED_JOBS)
