"""Run status aggregation in ``process_runs`` (reference: ``src/tests/_internal/server/background/
tasks/test_process_runs.py``): the run status from its replicas' latest job submissions (FAILED >
RUNNING > PROVISIONING > SUBMITTED > DONE), retry to PENDING on no-capacity / interruption, the
retry-duration limit, PENDING -> SUBMITTED after the resubmission delay, and multi-replica services
where one replica's failure is retried without leaving RUNNING."""

from __future__ import annotations

from datetime import timedelta
from typing import List
from unittest import mock

import pytest

from dstack_amd.core.models.runs import JobStatus, JobTerminationReason, RunSpec, RunStatus, RunTerminationReason
from dstack_amd.server.background.tasks import process_runs as pr
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import JobModel, ProjectModel, RunModel, UserModel
from dstack_amd.server.services import runs as runs_services
from dstack_amd.utils.common import get_current_datetime

RETRY = {"on_events": ["no-capacity", "interruption", "error"], "duration": "1h"}
JPD = ('{"backend": "aws", "instance_type": {"name": "i", "resources": {"cpus": 4, "memory_mib": 8192, '
       '"gpus": [], "spot": false}}, "instance_id": "i-1", "hostname": "1.1.1.1", "region": "us", "price": 1.0, '
       '"username": "ubuntu", "ssh_port": 22, "dockerized": true}')


def _run(conf: dict, status: RunStatus = RunStatus.SUBMITTED, retry=None) -> str:
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="main").one()
        user = s.query(UserModel).filter_by(name="admin").one()
        profile = {"name": "default"}
        if retry is not None:
            profile["retry"] = retry
        spec = RunSpec.model_validate({"run_name": "rr", "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                                       "configuration": conf, "profile": profile})
        run_id = runs_services.submit_run(s, project, user, spec).id
        s.get(RunModel, run_id).status = status.value
        return run_id


def _task(**kw):
    return {"type": "task", "commands": ["true"], **kw}


def _service(replicas=2):
    return {"type": "service", "commands": ["serve"], "port": 8000, "replicas": replicas}


def _set_jobs(run_id, *states):
    """states[i] = (JobStatus, termination reason or None, provisioned?) for replica i's job."""
    with session_scope() as s:
        jobs: List[JobModel] = sorted(s.query(JobModel).filter_by(run_id=run_id), key=lambda j: j.replica_num)
        for j, st in zip(jobs, states):
            status, reason, provisioned = (st + (None, None))[:3] if isinstance(st, tuple) else (st, None, None)
            j.status = status.value
            j.termination_reason = reason.value if reason else None
            if provisioned or status in (JobStatus.PROVISIONING, JobStatus.PULLING, JobStatus.RUNNING):
                j.job_provisioning_data = JPD
            if status.is_finished():
                j.finished_at = get_current_datetime()


def _process(run_id, at=None):
    with mock.patch.object(pr, "get_current_datetime", return_value=at or get_current_datetime()):
        with session_scope() as s:
            pr._process_run(s, run_id)
    with session_scope() as s:
        run = s.get(RunModel, run_id)
        return RunStatus(run.status), run.termination_reason, sorted(
            (j.replica_num, j.submission_num, j.status) for j in run.jobs)


@pytest.mark.parametrize("job_status,run_status", [
    (JobStatus.SUBMITTED, RunStatus.SUBMITTED),
    (JobStatus.PROVISIONING, RunStatus.PROVISIONING),
    (JobStatus.PULLING, RunStatus.PROVISIONING),  # keep provisioning while the image pulls
    (JobStatus.RUNNING, RunStatus.RUNNING),
])
def test_single_job_status_maps_to_run(db, job_status, run_status):
    rid = _run(_task())
    _set_jobs(rid, job_status)
    assert _process(rid)[0] == run_status


def test_running_to_done(db):
    rid = _run(_task(), RunStatus.RUNNING)
    _set_jobs(rid, (JobStatus.DONE, JobTerminationReason.DONE_BY_RUNNER, True))
    st, reason, _ = _process(rid)
    assert st == RunStatus.TERMINATING and reason == RunTerminationReason.ALL_JOBS_DONE.value


def test_failed_job_without_retry_terminates_run(db):
    rid = _run(_task(), RunStatus.RUNNING)
    _set_jobs(rid, (JobStatus.FAILED, JobTerminationReason.CONTAINER_EXITED_WITH_ERROR, True))
    st, reason, _ = _process(rid)
    assert st == RunStatus.TERMINATING and reason == RunTerminationReason.JOB_FAILED.value


def test_retry_running_to_pending_then_submitted(db):
    rid = _run(_task(), RunStatus.RUNNING, retry=RETRY)
    _set_jobs(rid, (JobStatus.FAILED, JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY, True))
    st, _, jobs = _process(rid)
    assert st == RunStatus.PENDING and len(jobs) == 1
    # resubmitted only after the retry delay
    assert _process(rid)[0] == RunStatus.PENDING
    st, _, jobs = _process(rid, at=get_current_datetime() + pr.RETRY_DELAY + timedelta(seconds=1))
    assert st == RunStatus.SUBMITTED
    assert jobs == [(0, 0, JobStatus.FAILED.value), (0, 1, JobStatus.SUBMITTED.value)]


def test_retry_limit_exceeded(db):
    rid = _run(_task(), RunStatus.RUNNING, retry={**RETRY, "duration": "10m"})
    _set_jobs(rid, (JobStatus.FAILED, JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY, True))
    st, reason, _ = _process(rid, at=get_current_datetime() + timedelta(hours=1))
    assert st == RunStatus.TERMINATING and reason == RunTerminationReason.RETRY_LIMIT_EXCEEDED.value


def test_no_capacity_not_retried_without_event(db):
    rid = _run(_task(), RunStatus.SUBMITTED, retry={"on_events": ["error"], "duration": "1h"})
    _set_jobs(rid, (JobStatus.FAILED, JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY))
    assert _process(rid)[0] == RunStatus.TERMINATING


# ---- multi-replica services ----------------------------------------------------------------------
@pytest.mark.parametrize("states,run_status", [
    ((JobStatus.SUBMITTED, JobStatus.PROVISIONING), RunStatus.PROVISIONING),  # provisioning if any
    ((JobStatus.PROVISIONING, JobStatus.RUNNING), RunStatus.RUNNING),  # running if any
])
def test_service_replicas_any_rule(db, states, run_status):
    rid = _run(_service())
    _set_jobs(rid, *states)
    assert _process(rid)[0] == run_status


def test_service_all_replicas_no_capacity_to_pending(db):
    rid = _run(_service(), RunStatus.SUBMITTED, retry=RETRY)
    _set_jobs(rid, (JobStatus.FAILED, JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY),
              (JobStatus.FAILED, JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY))
    assert _process(rid)[0] == RunStatus.PENDING


def test_service_some_no_capacity_keeps_running_and_retries_replica(db):
    rid = _run(_service(), RunStatus.RUNNING, retry=RETRY)
    _set_jobs(rid, JobStatus.RUNNING, (JobStatus.FAILED, JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY))
    st, _, jobs = _process(rid)
    assert st == RunStatus.RUNNING
    assert (1, 1, JobStatus.SUBMITTED.value) in jobs  # the failed replica got a new submission


def test_service_some_failed_without_retry_terminates(db):
    rid = _run(_service(), RunStatus.RUNNING)
    _set_jobs(rid, JobStatus.RUNNING, (JobStatus.FAILED, JobTerminationReason.CONTAINER_EXITED_WITH_ERROR, True))
    st, reason, _ = _process(rid)
    assert st == RunStatus.TERMINATING and reason == RunTerminationReason.JOB_FAILED.value


def test_pending_service_resubmits_every_replica(db):
    rid = _run(_service(), RunStatus.PENDING, retry=RETRY)
    _set_jobs(rid, (JobStatus.FAILED, JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY),
              (JobStatus.FAILED, JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY))
    st, _, jobs = _process(rid, at=get_current_datetime() + pr.RETRY_DELAY + timedelta(seconds=1))
    assert st == RunStatus.SUBMITTED
    assert [(r, n, js) for r, n, js in jobs if js == JobStatus.SUBMITTED.value] == [
        (0, 1, JobStatus.SUBMITTED.value), (1, 1, JobStatus.SUBMITTED.value)]


def test_terminating_run_terminates_its_jobs_then_finishes(db):
    """(reference ``test_terminate_run_jobs``) a run stopped by the user: its running job is moved
    to TERMINATING with the run's reason mapped; once the job is finished the run is too."""
    rid = _run(_task(), RunStatus.RUNNING)
    _set_jobs(rid, JobStatus.RUNNING)
    with session_scope() as s:
        run = s.get(RunModel, rid)
        run.status = RunStatus.TERMINATING.value
        run.termination_reason = RunTerminationReason.STOPPED_BY_USER.value
    with mock.patch("dstack_amd.server.services.jobs.stop_runner"):
        st, reason, jobs = _process(rid)
    assert st == RunStatus.TERMINATING and jobs == [(0, 0, "terminating")]
    with session_scope() as s:
        j = s.query(JobModel).filter_by(run_id=rid).one()
        assert j.termination_reason == JobTerminationReason.TERMINATED_BY_USER.value
        j.status = JobStatus.TERMINATED.value
    st, reason, _ = _process(rid)
    assert st == RunStatus.TERMINATED and reason == RunTerminationReason.STOPPED_BY_USER.value


# ---- gpu_util autoscaling through the DB ---------------------------------------------------------
def _gpu_util_service():
    return {"type": "service", "commands": ["serve"], "port": 8000, "replicas": "1..4",
            "scaling": {"metric": "gpu_util", "target": 70, "scale_up_delay": 60, "scale_down_delay": 300}}


def _util_samples(run_id, pct_by_replica, age_s: float = 0.0):
    """One amdsmi sample (8 GPUs at ``pct``) per running replica, ``age_s`` seconds old (wall clock:
    the metric reads the last 120 s of JobMetricsPoint rows, as process_metrics writes them)."""
    import json
    import time
    import uuid

    from dstack_amd.server.models import JobMetricsPoint

    ts = int((time.time() - age_s) * 1e6)
    with session_scope() as s:
        latest = {}
        for j in s.query(JobModel).filter_by(run_id=run_id):
            if j.replica_num not in latest or j.submission_num > latest[j.replica_num].submission_num:
                latest[j.replica_num] = j
        for r, pct in pct_by_replica.items():
            s.add(JobMetricsPoint(id=uuid.uuid4(), job_id=latest[r].id, timestamp_micro=ts, cpu_usage_micro=0,
                                  memory_usage_bytes=0, memory_working_set_bytes=0,
                                  gpus_memory_usage_bytes=json.dumps([0] * 8), gpus_util_percent=json.dumps([pct] * 8)))


def _process_scaling(run_id, at):
    from dstack_amd.server.services import services as services_services

    with mock.patch.object(services_services, "get_current_datetime", return_value=at):
        return _process(run_id, at)


def _active_replicas(run_id) -> List[int]:
    from dstack_amd.server.services import jobs as jobs_services

    with session_scope() as s:
        run = s.get(RunModel, run_id)
        groups = jobs_services.group_jobs_by_replica_latest(run.jobs)
        return sorted(r for r, js in groups.items()
                      if any(not JobStatus(j.status).is_finished() and j.status != JobStatus.TERMINATING.value
                             for j in js))


def _set_latest_running(run_id):
    with session_scope() as s:
        for j in s.query(JobModel).filter_by(run_id=run_id):
            if j.status == JobStatus.SUBMITTED.value:
                j.status = JobStatus.RUNNING.value
                j.job_provisioning_data = JPD


def test_gpu_util_autoscaling_through_job_metrics(db):
    """``scaling: {metric: gpu_util, target: 70}`` end to end at the reconciler level (reference
    services/services/autoscalers.py:75-108 for the RPS form; gpu_util is this build's amdsmi
    metric): JobMetricsPoint rows -> service_metric_value (mean util of the running replicas over
    the last 120 s) -> GPUUtilAutoscaler -> scale_run_replicas.  2 replicas at 95 % -> 3 once the
    scale-up delay has passed; at 20 % -> 1, not before the scale-down delay."""
    rid = _run(_gpu_util_service(), RunStatus.RUNNING)
    with session_scope() as s:
        runs_services.scale_run_replicas(s, s.get(RunModel, rid), 1)  # 2 replicas
    _set_latest_running(rid)
    t0 = get_current_datetime()
    assert _active_replicas(rid) == [0, 1]
    # no samples at all: nothing to scale on
    _process_scaling(rid, t0 + timedelta(minutes=2))
    assert _active_replicas(rid) == [0, 1]
    # a stale sample (older than 120 s) is ignored
    _util_samples(rid, {0: 95.0, 1: 95.0}, age_s=300)
    _process_scaling(rid, t0 + timedelta(minutes=2))
    assert _active_replicas(rid) == [0, 1]
    # hot: ceil(2 * 95 / 70) = 3, but not within the scale-up delay of the last replica start
    _util_samples(rid, {0: 95.0, 1: 95.0})
    _process_scaling(rid, t0 + timedelta(seconds=30))
    assert _active_replicas(rid) == [0, 1]
    _process_scaling(rid, t0 + timedelta(minutes=2))
    assert _active_replicas(rid) == [0, 1, 2]
    with session_scope() as s:
        assert s.get(RunModel, rid).desired_replica_count == 3
    _set_latest_running(rid)
    # one replica without samples does not drag the mean: 0 and 1 at 95 %, 2 unsampled -> stays
    _process_scaling(rid, t0 + timedelta(minutes=3))
    assert _active_replicas(rid) == [0, 1, 2]
    # cold: ceil(3 * 20 / 70) = 1; the scale-down delay (300 s) runs from the newest replica start
    _util_samples(rid, {0: 20.0, 1: 20.0, 2: 20.0})
    _process_scaling(rid, get_current_datetime() + timedelta(minutes=2))
    assert _active_replicas(rid) == [0, 1, 2]
    _process_scaling(rid, get_current_datetime() + timedelta(minutes=10))
    assert _active_replicas(rid) == [0]
    with session_scope() as s:
        run = s.get(RunModel, rid)
        stopped = [j for j in run.jobs if j.replica_num in (1, 2)]
        assert stopped and all(j.termination_reason == JobTerminationReason.SCALED_DOWN.value for j in stopped)
        assert run.desired_replica_count == 1 and RunStatus(run.status) == RunStatus.RUNNING
