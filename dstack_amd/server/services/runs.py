"""Runs service (reference: ``S/services/runs.py:273-1020``): plan, apply, submit, stop, delete,
model conversion, terminating-run handling, replica scaling and retry."""

from __future__ import annotations

import json
import logging
import re
import uuid
from datetime import datetime
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.common import ApplyAction
from dstack_amd.core.models.configurations import ServiceConfiguration, TaskConfiguration
from dstack_amd.core.models.profiles import CreationPolicy
from dstack_amd.core.models.runs import (
    Job,
    JobPlan,
    JobStatus,
    JobTerminationReason,
    Run,
    RunPlan,
    RunSpec,
    RunStatus,
    RunTerminationReason,
    ServiceSpec,
)
from dstack_amd.server import settings
from dstack_amd.server.background import scheduler
from dstack_amd.server.models import JobModel, ProjectModel, RunModel, UserModel
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.server.services import offers as offers_services
from dstack_amd.server.services import pools as pools_services
from dstack_amd.server.services import repos as repos_services
from dstack_amd.server.services.locking import db_advisory_lock, lockset
from dstack_amd.utils.common import generate_name, get_current_datetime

logger = logging.getLogger(__name__)

_RUN_NAME_RE = re.compile(r"^[a-z][a-z0-9-]{1,40}$")


def run_model_to_run(run: RunModel, include_jobs: bool = True, return_in_api: bool = False) -> Run:
    jobs: List[Job] = []
    if include_jobs:
        by_job: dict = {}
        for j in sorted(run.jobs, key=lambda j: (j.replica_num, j.job_num, j.submission_num)):
            key = (j.replica_num, j.job_num)
            if key not in by_job:
                by_job[key] = Job(job_spec=jobs_services.job_spec(j), job_submissions=[])
            by_job[key].job_spec = jobs_services.job_spec(j)
            by_job[key].job_submissions.append(jobs_services.job_model_to_job_submission(j))
        jobs = list(by_job.values())
    latest = None
    if run.jobs:
        latest_job = max(run.jobs, key=lambda j: (j.submitted_at, j.submission_num))
        latest = jobs_services.job_model_to_job_submission(latest_job)
    spec = RunSpec.model_validate_json(run.run_spec)
    cost = 0.0
    for j in run.jobs:
        jpd = jobs_services.job_jpd(j)
        if jpd is None:
            continue
        end = j.finished_at or get_current_datetime()
        cost += jpd.price * max(0.0, (end - j.submitted_at).total_seconds()) / 3600
    return Run(
        id=run.id, project_name=run.project.name, user=run.user.name, submitted_at=run.submitted_at,
        last_processed_at=run.last_processed_at, status=RunStatus(run.status),
        termination_reason=RunTerminationReason(run.termination_reason) if run.termination_reason else None,
        run_spec=spec, jobs=jobs, latest_job_submission=latest, cost=round(cost, 4),
        service=ServiceSpec.model_validate_json(run.service_spec) if run.service_spec else None,
        deleted=run.deleted,
    )


def list_user_runs(s: Session, user: UserModel, project_name: Optional[str] = None, repo_id: Optional[str] = None,
                   only_active: bool = False, limit: int = 100, prev_submitted_at: Optional[datetime] = None,
                   ascending: bool = False, username: Optional[str] = None,
                   prev_run_id: Optional[uuid.UUID] = None) -> List[Run]:
    """Runs of the projects the user sees (all for a global admin), newest first, as keyset pages:
    the next page starts after (``prev_submitted_at``, ``prev_run_id``) of the previous page's last
    run (reference ``S/services/runs.py:list_user_runs``).  ``repo_id`` needs ``project_name``;
    ``username`` keeps one user's runs."""
    from sqlalchemy import and_, or_

    from dstack_amd.server.services.projects import list_user_projects
    from dstack_amd.server.services.users import get_user_by_name

    if project_name is None and repo_id is not None:
        return []
    projects = list_user_projects(s, user)
    if project_name:
        projects = [p for p in projects if p.name == project_name]
    if not projects:
        return []
    q = select(RunModel).where(RunModel.project_id.in_([p.id for p in projects]), RunModel.deleted == False)  # noqa
    if repo_id is not None:
        q = q.where(RunModel.repo_id == repos_services.get_repo_or_error(s, projects[0], repo_id).id)
    if username is not None:
        runs_user = get_user_by_name(s, username)
        if runs_user is None:
            raise ResourceNotExistsError("User not found")
        q = q.where(RunModel.user_id == runs_user.id)
    if only_active:
        q = q.where(RunModel.status.notin_([st.value for st in RunStatus.finished_statuses()]))
    if prev_submitted_at is not None:
        after = RunModel.submitted_at > prev_submitted_at if ascending else RunModel.submitted_at < prev_submitted_at
        if prev_run_id is None:
            q = q.where(after)
        else:
            tie = RunModel.id > prev_run_id if ascending else RunModel.id < prev_run_id
            q = q.where(or_(after, and_(RunModel.submitted_at == prev_submitted_at, tie)))
    if ascending:
        q = q.order_by(RunModel.submitted_at.asc(), RunModel.id.asc())
    else:
        q = q.order_by(RunModel.submitted_at.desc(), RunModel.id.desc())
    return [run_model_to_run(r) for r in s.execute(q.limit(limit)).scalars()]


def get_run_model(s: Session, project: ProjectModel, run_name: Optional[str] = None,
                  run_id: Optional[uuid.UUID] = None) -> Optional[RunModel]:
    q = select(RunModel).where(RunModel.project_id == project.id)
    if run_id is not None:
        q = q.where(RunModel.id == run_id)
    else:
        q = q.where(RunModel.run_name == run_name, RunModel.deleted == False)  # noqa: E712
    return s.execute(q.order_by(RunModel.submitted_at.desc())).scalars().first()


def get_run(s: Session, project: ProjectModel, run_name: Optional[str] = None,
            run_id: Optional[uuid.UUID] = None) -> Optional[Run]:
    r = get_run_model(s, project, run_name, run_id)
    return run_model_to_run(r) if r else None


def _validate_run_spec(run_spec: RunSpec):
    if run_spec.run_name is not None and not _RUN_NAME_RE.match(run_spec.run_name):
        raise ServerClientError("Run name must be 2-41 chars of a-z, 0-9 and -, starting with a letter")
    from dstack_amd.server.services.docker import is_valid_docker_volume_target

    for mp in getattr(run_spec.configuration, "volumes", None) or []:
        if not is_valid_docker_volume_target(mp.path):
            raise ServerClientError(f"Invalid volume mount path: {mp.path}")
        if mp.path == "/workflow" or mp.path.startswith("/workflow/"):
            raise ServerClientError("Mounting volumes inside /workflow is not supported")


def get_plan(s: Session, project: ProjectModel, user: UserModel, run_spec: RunSpec, max_offers: int = 50) -> RunPlan:
    _validate_run_spec(run_spec)
    effective = run_spec.model_copy(deep=True)
    if effective.run_name is None:
        effective.run_name = "dry-run"
    current = None
    action = ApplyAction.CREATE
    if run_spec.run_name:
        cur = get_run_model(s, project, run_spec.run_name)
        if cur is not None and not RunStatus(cur.status).is_finished():
            current = run_model_to_run(cur)
            # UPDATE only when the change can be applied to the live run (replicas / scaling);
            # anything else is a CREATE the client must stop the active run for first
            if _updatable(RunSpec.model_validate_json(cur.run_spec), run_spec):
                action = ApplyAction.UPDATE
    profile = effective.merged_profile
    job_plans = []
    pool = pools_services.get_or_create_default_pool(s, project)
    instances = pools_services.list_project_instances(s, project)
    for spec in jobs_services.get_jobs_from_run_spec(effective, replica_num=0):
        multinode = spec.jobs_per_replica > 1
        pool_offers = [o for _, o in pools_services.filter_pool_instances(instances, profile, spec.requirements,
                                                                          multinode=multinode)]
        offers = pool_offers[:]
        if profile.creation_policy != CreationPolicy.REUSE:
            backend_offers = offers_services.get_offers_by_requirements(
                s, project, profile, spec.requirements, multinode=multinode, privileged=spec.privileged,
                instance_mounts=jobs_services.has_required_instance_mounts(spec),
            )
            offers += [o for _, o in backend_offers]
        job_plans.append(JobPlan(job_spec=spec, offers=offers[:max_offers], total_offers=len(offers),
                                 max_price=max((o.price for o in offers), default=None)))
    run_spec.run_name = run_spec.run_name  # plan keeps the user's (possibly None) name
    _ = pool
    return RunPlan(project_name=project.name, user=user.name, run_spec=run_spec, job_plans=job_plans,
                   current_resource=current, action=action)


def submit_run(s: Session, project: ProjectModel, user: UserModel, run_spec: RunSpec) -> Run:
    _validate_run_spec(run_spec)
    with db_advisory_lock(s, f"run_names_{project.id}"):
        if run_spec.run_name is None:
            for _ in range(20):
                name = generate_name()
                if get_run_model(s, project, name) is None:
                    run_spec.run_name = name
                    break
        else:
            existing = get_run_model(s, project, run_spec.run_name)
            if existing is not None:
                if not RunStatus(existing.status).is_finished():
                    raise ServerClientError(f"Run {run_spec.run_name} is already active")
                existing.deleted = True
        repo = repos_services.get_repo(s, project, run_spec.repo_id) if run_spec.repo_id else None
        if repo is None:
            # a virtual repo has no code to upload, so it needs no ``repos/init``; a remote or local
            # one must have been initialised (reference: RepoDoesNotExistError)
            if run_spec.repo_id and getattr(run_spec.repo_data, "repo_type", "virtual") != "virtual":
                raise ServerClientError(f"Repo {run_spec.repo_id} does not exist")
            repo = repos_services.get_or_create_virtual_repo(s, project, run_spec.repo_id or "none")
        now = get_current_datetime()
        conf = run_spec.configuration
        replicas = conf.replicas.min if isinstance(conf, ServiceConfiguration) else 1
        run = RunModel(id=uuid.uuid4(), project_id=project.id, user_id=user.id, repo_id=repo.id,
                       run_name=run_spec.run_name, submitted_at=now, last_processed_at=now,
                       status=RunStatus.SUBMITTED.value, run_spec=run_spec.model_dump_json(),
                       desired_replica_count=replicas)
        s.add(run)
        s.flush()
        secrets = jobs_services.get_job_secrets(s, project)
        for replica_num in range(replicas):
            for spec in jobs_services.get_jobs_from_run_spec(run_spec, replica_num, secrets):
                s.add(jobs_services.new_job_model(run, spec))
        if isinstance(conf, ServiceConfiguration):
            from dstack_amd.server.services.services import register_service

            register_service(s, run)
        s.flush()
        s.refresh(run)
    scheduler.wake(scheduler.SUBMITTED_JOBS, scheduler.RUNS)
    return run_model_to_run(run)


def apply_plan(s: Session, project: ProjectModel, user: UserModel, run_spec: RunSpec,
               current_resource: Optional[Run] = None, force: bool = False) -> Run:
    """Create, or update in place when only replica/scaling params changed (``apply_plan``)."""
    if run_spec.run_name:
        cur = get_run_model(s, project, run_spec.run_name)
        if cur is not None and not RunStatus(cur.status).is_finished():
            cur_spec = RunSpec.model_validate_json(cur.run_spec)
            if not force and current_resource is not None and current_resource.id != cur.id:
                raise ServerClientError("The run changed since the plan was made; re-plan or use --force")
            if not _updatable(cur_spec, run_spec):
                # the client stops the run and waits for it to finish before re-applying
                raise ServerClientError("Cannot override active run. Stop the run first.")
            cur.run_spec = run_spec.model_dump_json()
            conf = run_spec.configuration
            if isinstance(conf, ServiceConfiguration):
                cur.desired_replica_count = max(conf.replicas.min, min(conf.replicas.max, cur.desired_replica_count))
            s.flush()
            scheduler.wake(scheduler.RUNS)
            return run_model_to_run(cur)
    return submit_run(s, project, user, run_spec)


# an active run is updated in place only when it is a service and nothing but these changed
# (reference ``S/services/runs.py:_check_can_update_run_spec``): new code and replica-count /
# autoscaling / prefix-stripping settings; anything else needs the run stopped and resubmitted
_UPDATABLE_SPEC = {"repo_code_hash", "configuration"}
_UPDATABLE = {"replicas", "scaling", "strip_prefix"}


def _changed(a: dict, b: dict) -> set:
    return {k for k in set(a) | set(b) if a.get(k) != b.get(k)}


def _updatable(old: RunSpec, new: RunSpec) -> bool:
    if old.configuration.type != "service" or new.configuration.type != "service":
        return False
    spec_diff = _changed(old.model_dump(mode="json"), new.model_dump(mode="json"))
    if not spec_diff <= _UPDATABLE_SPEC:
        return False
    return _changed(old.configuration.model_dump(mode="json"), new.configuration.model_dump(mode="json")) <= _UPDATABLE


def stop_runs(s: Session, project: ProjectModel, runs_names: List[str], abort: bool):
    """Mark the runs TERMINATING (``S/services/runs.py:stop_runs``).

    The runs are held in the background processor's ``runs`` lockset (and row-locked on Postgres)
    and the change is committed before they are released: otherwise a ``process_runs`` pass that
    loaded a run just before the stop (e.g. while it was provisioning) writes its own status
    transition back over TERMINATING, and the run keeps running with a termination reason set."""
    reason = RunTerminationReason.ABORTED_BY_USER if abort else RunTerminationReason.STOPPED_BY_USER
    runs = [r for r in (get_run_model(s, project, name) for name in runs_names) if r is not None]
    with lockset("runs").hold([r.id for r in runs], timeout=60.0):
        for run in runs:
            s.refresh(run, with_for_update=True)  # the state the last background pass committed
            if RunStatus(run.status).is_finished():
                continue
            run.status = RunStatus.TERMINATING.value
            run.termination_reason = reason.value
            run.last_processed_at = get_current_datetime()
        s.commit()
    scheduler.wake(scheduler.RUNS)


def delete_runs(s: Session, project: ProjectModel, runs_names: List[str]):
    for name in runs_names:
        run = get_run_model(s, project, name)
        if run is None:
            continue
        if not RunStatus(run.status).is_finished():
            raise ServerClientError(f"Run {name} is not finished; stop it first")
        run.deleted = True


def process_terminating_run(s: Session, run: RunModel):
    """Stop every unfinished job of a TERMINATING run; finish the run once all jobs are done
    (``S/services/runs.py:876-922``)."""
    reason = RunTerminationReason(run.termination_reason)
    job_reason = reason.to_job_termination_reason()
    unfinished = False
    for job in run.jobs:
        st = JobStatus(job.status)
        if st.is_finished():
            continue
        unfinished = True
        if st == JobStatus.TERMINATING:
            continue
        if st == JobStatus.RUNNING and job_reason != JobTerminationReason.ABORTED_BY_USER:
            jobs_services.stop_runner(s, job)
            jobs_services.terminate_job(job, job_reason, delay=True)
        else:
            jobs_services.terminate_job(job, job_reason, delay=False)
    if not unfinished:
        run.status = reason.to_status().value
        if isinstance(RunSpec.model_validate_json(run.run_spec).configuration, ServiceConfiguration):
            from dstack_amd.server.services.services import unregister_service

            unregister_service(s, run)
    scheduler.wake(scheduler.TERMINATING_JOBS)


def _replica_importance(jobs: List[JobModel]) -> Optional[int]:
    """None for an inactive replica (any job terminating or finished), else how costly stopping it
    is: 0 still submitted, 1 provisioning or pulling, 2 running."""
    statuses = {JobStatus(j.status) for j in jobs}
    if JobStatus.TERMINATING in statuses or any(st.is_finished() for st in statuses):
        return None
    if JobStatus.SUBMITTED in statuses:
        return 0
    if statuses & {JobStatus.PROVISIONING, JobStatus.PULLING}:
        return 1
    return 2


def scale_run_replicas(s: Session, run: RunModel, replicas_diff: int):
    """Scale a service by ``replicas_diff`` replicas (reference ``services/runs.py:scale_run_replicas``).

    Down: the least important active replicas stop first (submitted before provisioning before
    running; among equals the highest replica number), never below ``replicas.min``.  Up: finished
    replicas are re-submitted first, then new replica numbers are added, never above ``replicas.max``."""
    if replicas_diff == 0:
        return
    spec = RunSpec.model_validate_json(run.run_spec)
    conf = spec.configuration
    groups = jobs_services.group_jobs_by_replica_latest(run.jobs)
    active, inactive = [], []
    for r, js in groups.items():
        imp = _replica_importance(js)
        (inactive if imp is None else active).append((imp, r, js))
    active.sort(key=lambda t: (-t[0], t[1]))  # most important first, then lower replica number
    lo = conf.replicas.min if isinstance(conf, ServiceConfiguration) else 0
    hi = conf.replicas.max if isinstance(conf, ServiceConfiguration) else None
    if replicas_diff < 0:
        if len(active) + replicas_diff < (lo or 0):
            raise ServerClientError("Can't scale down below the minimum number of replicas")
        for _, _, js in reversed(active[replicas_diff:]):
            for j in js:
                if JobStatus(j.status).is_finished() or j.status == JobStatus.TERMINATING.value:
                    continue
                if j.status == JobStatus.RUNNING.value:
                    jobs_services.stop_runner(s, j)
                jobs_services.terminate_job(j, JobTerminationReason.SCALED_DOWN)
        scheduler.wake(scheduler.TERMINATING_JOBS)
        return
    if hi is not None and len(active) + replicas_diff > hi:
        raise ServerClientError("Can't scale up above the maximum number of replicas")
    scheduled = 0
    for _, _, js in sorted(inactive, key=lambda t: t[1]):  # re-run finished replicas first
        if scheduled == replicas_diff:
            break
        retry_run_replica_jobs(s, run, js, only_failed=False)
        scheduled += 1
    secrets = jobs_services.get_job_secrets(s, run.project)
    next_replica = max(groups.keys(), default=-1) + 1
    for r in range(next_replica, next_replica + replicas_diff - scheduled):
        for js in jobs_services.get_jobs_from_run_spec(spec, r, secrets):
            s.add(jobs_services.new_job_model(run, js, submission_num=0))
    s.flush()
    scheduler.wake(scheduler.SUBMITTED_JOBS)


def retry_run_replica_jobs(s: Session, run: RunModel, latest_jobs: List[JobModel], only_failed: bool):
    """New submissions for a replica's jobs (``retry_run_replica_jobs``)."""
    spec = RunSpec.model_validate_json(run.run_spec)
    secrets = jobs_services.get_job_secrets(s, run.project)
    for old in latest_jobs:
        if only_failed and JobStatus(old.status) not in (JobStatus.FAILED, JobStatus.TERMINATED, JobStatus.ABORTED):
            continue
        for js in jobs_services.get_jobs_from_run_spec(spec, old.replica_num, secrets):
            if js.job_num == old.job_num:
                s.add(jobs_services.new_job_model(run, js, submission_num=old.submission_num + 1))
    s.flush()
    scheduler.wake(scheduler.SUBMITTED_JOBS)


def is_multinode(run_spec: RunSpec) -> bool:
    c = run_spec.configuration
    return isinstance(c, TaskConfiguration) and c.nodes > 1


def get_run_by_name_or_error(s: Session, project: ProjectModel, name: str) -> RunModel:
    r = get_run_model(s, project, name)
    if r is None:
        raise ResourceNotExistsError(f"Run {name} not found")
    return r


def settings_snapshot() -> dict:
    return {"event_driven": settings.SERVER_EVENT_DRIVEN}


__all__ = [
    "get_plan", "apply_plan", "submit_run", "stop_runs", "delete_runs", "list_user_runs", "get_run",
    "run_model_to_run", "process_terminating_run", "scale_run_replicas", "retry_run_replica_jobs", "json",
]
