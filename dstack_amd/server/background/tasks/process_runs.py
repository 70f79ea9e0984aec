"""Run status aggregation, retry and service autoscaling (reference:
``S/background/tasks/process_runs.py:46-414``).

Per replica (latest submission of each job): DONE / RUNNING / PROVISIONING / SUBMITTED / FAILED;
a failed job is retried (the whole replica gets new submissions) when its termination reason
maps to a ``retry.on_events`` event and the retry duration is not exceeded; otherwise the run
fails.  Run status = FAILED > RUNNING > PROVISIONING > SUBMITTED > DONE(all) > PENDING.
PENDING runs (waiting for capacity) are resubmitted after ``RETRY_DELAY``.
"""

from __future__ import annotations

import logging
from datetime import timedelta
from typing import List, Optional, Set, Tuple

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ServerClientError
from dstack_amd.core.models.configurations import ServiceConfiguration
from dstack_amd.core.models.profiles import RetryEvent
from dstack_amd.core.models.runs import JobStatus, JobTerminationReason, RunSpec, RunStatus, RunTerminationReason
from dstack_amd.server.background import scheduler
from dstack_amd.server.background.common import claim_and_process
from dstack_amd.server.models import JobModel, RunModel
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.server.services import runs as runs_services
from dstack_amd.server.services import services as services_services
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)
RETRY_DELAY = timedelta(seconds=15)

_ERROR_REASONS = {
    JobTerminationReason.CONTAINER_EXITED_WITH_ERROR, JobTerminationReason.CREATING_CONTAINER_ERROR,
    JobTerminationReason.EXECUTOR_ERROR, JobTerminationReason.GATEWAY_ERROR,
    JobTerminationReason.WAITING_INSTANCE_LIMIT_EXCEEDED, JobTerminationReason.WAITING_RUNNER_LIMIT_EXCEEDED,
    JobTerminationReason.PORTS_BINDING_FAILED, JobTerminationReason.GPU_HEALTH_CHECK_FAILED,
}


def process_runs(batch: int = 10) -> bool:
    def select_ids(s: Session):
        return s.execute(select(RunModel.id).where(RunModel.status.notin_([x.value for x in
                                                                           RunStatus.finished_statuses()]))
                         .where(RunModel.deleted == False)  # noqa: E712
                         .order_by(RunModel.last_processed_at).limit(batch * 4)).scalars()

    return claim_and_process("runs", select_ids, _process_run, batch)


def _process_run(s: Session, run_id):
    run = s.get(RunModel, run_id)
    if run is None:
        return
    s.refresh(run)
    if RunStatus(run.status).is_finished():
        return  # finished between selection and claim (another pass finished it): nothing to do
    if run.status == RunStatus.TERMINATING.value:
        runs_services.process_terminating_run(s, run)
    elif run.status == RunStatus.PENDING.value:
        _process_pending(s, run)
    else:
        _process_active(s, run)
    run.last_processed_at = get_current_datetime()


def _retry_duration(run: RunModel, job: JobModel) -> Optional[timedelta]:
    """None = not retryable; else the time spent retrying so far (``_should_retry_job``)."""
    spec = jobs_services.job_spec(job)
    if spec.retry is None:
        return None
    reason = JobTerminationReason(job.termination_reason) if job.termination_reason else None
    same = [j for j in run.jobs if j.replica_num == job.replica_num and j.job_num == job.job_num]
    provisioned = [j for j in same if j.job_provisioning_data is not None]
    last_prov = max(provisioned, key=lambda j: j.submission_num) if provisioned else None
    now = get_current_datetime()
    if reason == JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY and last_prov is None and \
            RetryEvent.NO_CAPACITY in spec.retry.on_events:
        return now - run.submitted_at
    if last_prov is None:
        return None
    lp_reason = JobTerminationReason(last_prov.termination_reason) if last_prov.termination_reason else None
    if lp_reason == JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY and RetryEvent.INTERRUPTION in spec.retry.on_events:
        return now - last_prov.last_processed_at
    if lp_reason in _ERROR_REASONS and RetryEvent.ERROR in spec.retry.on_events:
        return now - last_prov.last_processed_at
    if reason == JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY and RetryEvent.NO_CAPACITY in spec.retry.on_events:
        return now - run.submitted_at
    return None


def _process_active(s: Session, run: RunModel):
    run_spec = RunSpec.model_validate_json(run.run_spec)
    statuses: Set[RunStatus] = set()
    reasons: Set[RunTerminationReason] = set()
    to_retry: List[Tuple[int, List[JobModel]]] = []
    replicas_info: List[services_services.ReplicaInfo] = []
    for replica_num, jobs in jobs_services.group_jobs_by_replica_latest(run.jobs).items():
        rstat: Set[RunStatus] = set()
        needs_retry = False
        active = True
        for j in jobs:
            if run.fleet_id is None and j.instance is not None and j.instance.fleet_id is not None:
                run.fleet_id = j.instance.fleet_id
            st = JobStatus(j.status)
            tr = JobTerminationReason(j.termination_reason) if j.termination_reason else None
            if st == JobStatus.DONE or (st == JobStatus.TERMINATING and tr == JobTerminationReason.DONE_BY_RUNNER):
                rstat.add(RunStatus.DONE)
                active = False
            elif tr == JobTerminationReason.SCALED_DOWN:
                active = False
            elif st == JobStatus.RUNNING:
                rstat.add(RunStatus.RUNNING)
            elif st in (JobStatus.PROVISIONING, JobStatus.PULLING):
                rstat.add(RunStatus.PROVISIONING)
            elif st == JobStatus.SUBMITTED:
                rstat.add(RunStatus.SUBMITTED)
            elif st == JobStatus.FAILED or (st == JobStatus.TERMINATING and tr not in (
                    JobTerminationReason.DONE_BY_RUNNER, JobTerminationReason.SCALED_DOWN)):
                dur = _retry_duration(run, j)
                spec = jobs_services.job_spec(j)
                if dur is None:
                    rstat.add(RunStatus.FAILED)
                    reasons.add(RunTerminationReason.JOB_FAILED)
                elif spec.retry is not None and dur > timedelta(seconds=spec.retry.duration):
                    rstat.add(RunStatus.FAILED)
                    reasons.add(RunTerminationReason.RETRY_LIMIT_EXCEEDED)
                else:
                    needs_retry = True
        if RunStatus.FAILED in rstat:
            statuses.add(RunStatus.FAILED)
        else:
            if needs_retry:
                to_retry.append((replica_num, jobs))
            else:
                statuses.update(rstat)
        if active:
            replicas_info.append(services_services.ReplicaInfo(True, min(j.submitted_at for j in jobs)))
        else:
            replicas_info.append(services_services.ReplicaInfo(False, max(j.last_processed_at for j in jobs)))

    reason: Optional[RunTerminationReason] = None
    if RunStatus.FAILED in statuses:
        new = RunStatus.TERMINATING
        reason = RunTerminationReason.JOB_FAILED if RunTerminationReason.JOB_FAILED in reasons \
            else RunTerminationReason.RETRY_LIMIT_EXCEEDED
    elif RunStatus.RUNNING in statuses:
        new = RunStatus.RUNNING
    elif RunStatus.PROVISIONING in statuses:
        new = RunStatus.PROVISIONING
    elif RunStatus.SUBMITTED in statuses:
        new = RunStatus.SUBMITTED
    elif RunStatus.DONE in statuses and not to_retry:
        new = RunStatus.TERMINATING
        reason = RunTerminationReason.ALL_JOBS_DONE
    elif not statuses and not to_retry and isinstance(run_spec.configuration, ServiceConfiguration):
        new = RunStatus.RUNNING if run.status == RunStatus.RUNNING.value else RunStatus.SUBMITTED  # scaled to 0
    else:
        new = RunStatus.PENDING

    if new == RunStatus.PENDING:
        for _, jobs in to_retry:
            for j in jobs:
                if not JobStatus(j.status).is_finished() and j.status != JobStatus.TERMINATING.value:
                    jobs_services.terminate_job(j, JobTerminationReason.TERMINATED_BY_SERVER, delay=False)
    if new not in (RunStatus.TERMINATING, RunStatus.PENDING):
        for _, jobs in to_retry:
            runs_services.retry_run_replica_jobs(s, run, jobs, only_failed=False)
        conf = run_spec.configuration
        if isinstance(conf, ServiceConfiguration):
            scaler = services_services.get_service_scaler(conf)
            metric = services_services.service_metric_value(s, run, conf)
            diff = scaler.scale(replicas_info, metric)
            if diff != 0:
                s.flush()
                s.refresh(run)
                run.desired_replica_count = sum(1 for r in replicas_info if r.active) + diff
                try:
                    runs_services.scale_run_replicas(s, run, diff)
                except ServerClientError as e:  # the scaler's view of active replicas lagged ours
                    logger.warning("run %s: not scaling by %d: %s", run.run_name, diff, e)
    if run.status != new.value:
        logger.info("run %s: %s -> %s", run.run_name, run.status, new.value)
        run.status = new.value
        run.termination_reason = reason.value if reason else None
        if new == RunStatus.TERMINATING:
            scheduler.wake(scheduler.RUNS)


def _process_pending(s: Session, run: RunModel):
    groups = jobs_services.group_jobs_by_replica_latest(run.jobs)
    finished = [j.finished_at for js in groups.values() for j in js if j.finished_at is not None]
    if any(not JobStatus(j.status).is_finished() for js in groups.values() for j in js):
        return  # wait for the failed replica's jobs to terminate
    if finished and get_current_datetime() - max(finished) < RETRY_DELAY:
        return
    for _, jobs in groups.items():
        if all(JobStatus(j.status).is_finished() for j in jobs):
            runs_services.retry_run_replica_jobs(s, run, jobs, only_failed=False)
    run.status = RunStatus.SUBMITTED.value
    run.resubmission_attempt = (run.resubmission_attempt or 0) + 1
    scheduler.wake(scheduler.SUBMITTED_JOBS)
