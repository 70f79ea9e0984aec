"""PROVISIONING -> PULLING -> RUNNING, and the running-job pull loop (reference:
``S/background/tasks/process_running_jobs.py:61-728``).

Cold-start path differences from the reference: the shim task and the runner submission happen
in the same pass when the agents are ready (no extra tick per stage); for the ``process`` shim
driver the runner is up in ~10 ms, so a job goes SUBMITTED -> RUNNING in one or two reconciler
passes.  Every stage is stamped into ``job.timings`` (cold-start instrumentation).
"""

from __future__ import annotations

import logging
import time
from datetime import timedelta
from typing import Dict, List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.backends.base import DSTACK_RUNNER_HTTP_PORT
from dstack_amd.core.errors import ResourceBusyError, RunnerError, ServerClientError, SSHError
from dstack_amd.core.models.common import NetworkMode
from dstack_amd.core.models.configurations import ServiceConfiguration
from dstack_amd.core.models.instances import InstanceStatus
from dstack_amd.core.models.runs import (
    ClusterInfo,
    JobStatus,
    JobTerminationReason,
    RunSpec,
    RunStatus,
)
from dstack_amd.core.models.volumes import InstanceMountPoint, VolumeMountPoint
from dstack_amd.server import settings
from dstack_amd.server.background import scheduler
from dstack_amd.server.background.common import claim_and_process
from dstack_amd.server.models import InstanceModel, JobModel, RunModel
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.server.services import logs as logs_services
from dstack_amd.server.services import repos as repos_services
from dstack_amd.server.services.runner.client import get_runner_client, get_shim_client
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)

ACTIVE = (JobStatus.PROVISIONING.value, JobStatus.PULLING.value, JobStatus.RUNNING.value)
PROVISIONING_TIMEOUT = timedelta(minutes=20)
# In-claim wait for an agent that is about to be ready (the process driver starts a task and its
# runner in ~10 ms): bounded so one slow host delays the rest of its batch by at most this much;
# after it the pass returns and re-queues the job with wake_later instead of sleeping.
AGENT_WAIT = 0.1
AGENT_RECHECK = 0.05


def process_running_jobs(batch: int = 5) -> bool:
    def select_ids(s: Session):
        return s.execute(select(JobModel.id).where(JobModel.status.in_(ACTIVE))
                         .order_by(JobModel.last_processed_at).limit(batch * 4)).scalars()

    return claim_and_process("jobs", select_ids, _process_job, batch)


def _process_job(s: Session, job_id):
    job = s.get(JobModel, job_id)
    if job is None or job.status not in ACTIVE:
        return
    run: RunModel = job.run
    if run.status == RunStatus.TERMINATING.value:
        return
    if job.status == JobStatus.PROVISIONING.value:
        _process_provisioning(s, run, job)
    if job.status == JobStatus.PULLING.value:
        _process_pulling(s, run, job)
    elif job.status == JobStatus.RUNNING.value:
        _process_running(s, run, job)
    job.last_processed_at = get_current_datetime()


def _cluster_info(run: RunModel, job: JobModel) -> Optional[ClusterInfo]:
    spec = jobs_services.job_spec(job)
    replica = [j for j in run.jobs if j.replica_num == job.replica_num]
    latest: Dict[int, JobModel] = {}
    for j in replica:
        if j.job_num not in latest or j.submission_num > latest[j.job_num].submission_num:
            latest[j.job_num] = j
    ips: List[str] = []
    for n in range(spec.jobs_per_replica):
        j = latest.get(n)
        jpd = jobs_services.job_jpd(j) if j else None
        if jpd is None or not (jpd.internal_ip or jpd.hostname):
            return None
        ips.append(jpd.internal_ip or jpd.hostname)
    jrd = jobs_services.job_jrd(job)
    gpus = 0
    if jrd and jrd.offer:
        gpus = len(jrd.offer.instance.resources.gpus)
    if jrd and jrd.gpu_indices is not None:
        gpus = len(jrd.gpu_indices)
    return ClusterInfo(job_ips=ips, master_job_ip=ips[0], gpus_per_job=gpus)


def _attach_volumes(s: Session, run: RunModel, job: JobModel) -> bool:
    """Attach the job's network volumes once its instance is up (``JobRuntimeData.volume_names``
    records them); a volume error fails the job with ``VOLUME_ERROR``, a volume held by another
    job's attach transaction is retried on a later pass."""
    from dstack_amd.server.services.jobs import volumes as job_volumes

    spec = jobs_services.job_spec(job)
    jrd = jobs_services.job_jrd(job)
    if jrd is None or jrd.volume_names is not None or not job_volumes.volume_mount_points(spec):
        return True
    inst = s.get(InstanceModel, job.instance_id) if job.instance_id is not None else None
    if inst is None:
        return True
    try:
        vols = job_volumes.get_job_configured_volumes(s, run.project, spec)
        job_volumes.check_can_attach_job_volumes(vols)
        jrd.volume_names = job_volumes.attach_job_volumes(s, job, inst, vols)
    except ResourceBusyError as e:
        logger.info("%s: %s; retrying", job.job_name, e)
        s.rollback()  # undo a partial attach of this pass (and release its volume locks)
        return False
    except ServerClientError as e:
        jobs_services.terminate_job(job, JobTerminationReason.VOLUME_ERROR, str(e), delay=False)
        scheduler.wake(scheduler.TERMINATING_JOBS)
        return False
    job.job_runtime_data = jrd.model_dump_json()
    return True


def _task_body(run: RunModel, job: JobModel, s: Optional[Session] = None) -> dict:
    spec = jobs_services.job_spec(job)
    jrd = jobs_services.job_jrd(job)
    run_spec = RunSpec.model_validate_json(run.run_spec)
    conf = run_spec.configuration
    gpu_req = conf.resources.gpu
    n_gpu = 0
    if gpu_req is not None and (gpu_req.count.max or 0) > 0 and jrd and jrd.offer:
        n_gpu = len(jrd.offer.instance.resources.gpus)
    shm = conf.resources.shm_size
    volume_mounts, instance_mounts = [], []
    for mp in spec.mount_points():
        if isinstance(mp, VolumeMountPoint):
            volume_mounts.append({"name": mp.name if isinstance(mp.name, str) else mp.name[0], "path": mp.path})
        elif isinstance(mp, InstanceMountPoint):
            instance_mounts.append({"instance_path": mp.instance_path, "path": mp.path, "optional": mp.optional})
    ports = [a.port for a in (spec.app_specs or [])]
    if isinstance(conf, ServiceConfiguration):
        ports.append(conf.port.container_port)
    keys = [run.project.ssh_public_key.strip()]
    if run_spec.ssh_key_pub:
        keys.append(run_spec.ssh_key_pub.strip())
    body = {
        "id": str(job.id), "name": job.job_name, "image_name": spec.image_name,
        "container_user": str(spec.user) if spec.user else "", "privileged": spec.privileged,
        "gpu": n_gpu, "gpu_indices": (jrd.gpu_indices or []) if jrd else [],
        "cpu": jrd.cpu if jrd and jrd.cpu else 0, "memory": int((jrd.memory or 0) * 2**30) if jrd else 0,
        "shm_size": int(shm * 2**30) if shm else 0,
        "network_mode": jrd.network_mode.value if jrd else "host",
        "volumes": _volume_specs(s, job, jrd), "volume_mounts": volume_mounts, "instance_mounts": instance_mounts,
        "container_ssh_keys": keys, "ports": ports,
        "host_ssh_user": "", "host_ssh_keys": [],
    }
    if spec.registry_auth:
        body["registry_username"] = spec.registry_auth.username
        body["registry_password"] = spec.registry_auth.password
    return body


def _volume_specs(s: Optional[Session], job: JobModel, jrd) -> list:
    if s is None or jrd is None or not jrd.volume_names:
        return []
    from dstack_amd.server.services.jobs.volumes import shim_volume_specs

    return shim_volume_specs(s, job, jrd.volume_names)


def _process_provisioning(s: Session, run: RunModel, job: JobModel):
    jpd = jobs_services.job_jpd(job)
    if jpd is None or not jpd.hostname:
        return  # process_instances fills the hostname when the cloud reports it
    if job.instance_id is not None:
        inst = s.get(InstanceModel, job.instance_id)
        if inst is not None and inst.status == InstanceStatus.PROVISIONING.value:
            return  # wait for the shim healthcheck in process_instances
    if _cluster_info(run, job) is None:
        return  # multinode: wait until every job of the replica has an address
    project = run.project
    if not jpd.dockerized:
        job.status = JobStatus.PULLING.value  # container backends: the runner *is* the container
        jobs_services.mark_timing(job, "pulling")
        return
    if not _attach_volumes(s, run, job):
        return
    try:
        shim = get_shim_client(jpd, project.ssh_private_key)
        shim.submit_task(_task_body(run, job, s))
    except (SSHError, RunnerError, Exception) as e:  # noqa: BLE001
        logger.info("%s: shim not reachable yet: %s", job.job_name, e)
        if get_current_datetime() - job.submitted_at > PROVISIONING_TIMEOUT:
            jobs_services.terminate_job(job, JobTerminationReason.WAITING_INSTANCE_LIMIT_EXCEEDED, str(e), delay=False)
            scheduler.wake(scheduler.TERMINATING_JOBS)
        return
    job.status = JobStatus.PULLING.value
    jobs_services.mark_timing(job, "pulling")


def _process_pulling(s: Session, run: RunModel, job: JobModel):
    jpd = jobs_services.job_jpd(job)
    project = run.project
    if jpd.dockerized:
        shim = get_shim_client(jpd, project.ssh_private_key)
        task = None
        deadline = time.monotonic() + AGENT_WAIT
        while True:
            try:
                task = shim.get_task(str(job.id))
            except Exception as e:  # noqa: BLE001
                logger.info("%s: shim get_task failed: %s", job.job_name, e)
                _runner_unreachable(job, f"shim: {e}")  # host gone while pulling: interrupted after a grace
                return
            if task is None:
                job.status = JobStatus.PROVISIONING.value  # shim lost the task (restart): resubmit
                return
            if task["status"] in ("running", "terminated") or time.monotonic() > deadline:
                break
            time.sleep(0.01)
        if task["status"] == "terminated":
            reason = task.get("termination_reason") or ""
            jr = JobTerminationReason.CREATING_CONTAINER_ERROR
            try:
                jr = JobTerminationReason(reason)
            except ValueError:
                pass
            jobs_services.terminate_job(job, jr, task.get("termination_message"), delay=False)
            scheduler.wake(scheduler.TERMINATING_JOBS)
            return
        if task["status"] != "running":
            scheduler.wake_later(AGENT_RECHECK, scheduler.RUNNING_JOBS)  # pulling an image: check again soon
            return
        job.remove_at = None
        jrd = jobs_services.job_jrd(job)
        ports = {int(p["container"]): int(p["host"]) for p in task.get("ports") or []}
        if task.get("runner_port"):
            ports[DSTACK_RUNNER_HTTP_PORT] = int(task["runner_port"])
        if jrd is not None and jrd.network_mode == NetworkMode.BRIDGE and DSTACK_RUNNER_HTTP_PORT not in ports:
            # bridge network: the runner is reachable only through its published port; not mapped yet
            scheduler.wake_later(AGENT_RECHECK, scheduler.RUNNING_JOBS)
            return
        jobs_services.mark_timing(job, "container_running")
        if jrd is not None:
            jrd.ports = ports or None
            if task.get("gpus") is not None and not jrd.gpu_indices:
                jrd.gpu_indices = [int(x) for x in task["gpus"]]
            job.job_runtime_data = jrd.model_dump_json()
    _submit_to_runner(s, run, job)


def _submit_to_runner(s: Session, run: RunModel, job: JobModel):
    jpd = jobs_services.job_jpd(job)
    jrd = jobs_services.job_jrd(job)
    project = run.project
    try:
        runner = get_runner_client(jpd, jrd, project.ssh_private_key)
    except SSHError as e:
        logger.info("%s: runner tunnel failed: %s", job.job_name, e)
        return
    deadline = time.monotonic() + AGENT_WAIT
    while runner.healthcheck() is None:
        if time.monotonic() > deadline:
            if get_current_datetime() - job.submitted_at > timedelta(seconds=settings.DEFAULT_RUNNER_TIMEOUT):
                jobs_services.terminate_job(job, JobTerminationReason.WAITING_RUNNER_LIMIT_EXCEEDED, delay=False)
                scheduler.wake(scheduler.TERMINATING_JOBS)
            else:
                scheduler.wake_later(AGENT_RECHECK, scheduler.RUNNING_JOBS)
            return
        time.sleep(0.01)
    run_spec = RunSpec.model_validate_json(run.run_spec)
    cluster = _cluster_info(run, job)
    repo = run.repo
    code = repos_services.get_code_blob(s, project, repo, run_spec.repo_code_hash)
    repo_data = run_spec.repo_data.model_dump(mode="json") if run_spec.repo_data else {"repo_type": repo.type}
    creds = repos_services.get_repo_creds(s, repo, run.user_id)
    secrets = jobs_services.get_job_secrets(s, project)
    try:
        runner.submit_job(run_spec, run.run_name, repo_data, jobs_services.job_spec(job), cluster, secrets, creds)
        runner.upload_code(code)
        runner.run_job()
    except Exception as e:  # noqa: BLE001
        logger.warning("%s: runner submit failed: %s", job.job_name, e)
        return
    job.status = JobStatus.RUNNING.value
    job.runner_timestamp = 0
    jobs_services.mark_timing(job, "running")
    if isinstance(run_spec.configuration, ServiceConfiguration):
        from dstack_amd.server.services.services import register_replica

        register_replica(s, run, job)
    scheduler.wake(scheduler.RUNS, scheduler.RUNNING_JOBS)


def _process_running(s: Session, run: RunModel, job: JobModel):
    jpd = jobs_services.job_jpd(job)
    jrd = jobs_services.job_jrd(job)
    try:
        runner = get_runner_client(jpd, jrd, run.project.ssh_private_key)
        resp = runner.pull(job.runner_timestamp or 0)
    except Exception as e:  # noqa: BLE001
        _runner_unreachable(job, str(e))
        return
    job.remove_at = None  # runner reachable again: clear the unreachable marker
    if resp.get("gpu_probe") and job.instance is not None:
        _record_gpu_probe(job, resp["gpu_probe"])
    if resp.get("rccl_preflight") and job.instance is not None:
        _record_rccl_preflight(job, resp["rccl_preflight"])
    if resp.get("job_logs") or resp.get("runner_logs"):
        logs_services.write_job_logs(run.project.name, run.run_name, str(job.id), resp)
        if resp.get("job_logs"):
            # the runner's own clock: when the workload printed, not when we polled
            first = resp["job_logs"][0].get("timestamp")
            jobs_services.mark_timing(job, "first_log", first / 1000.0 if first else None)
    job.runner_timestamp = int(resp.get("last_updated") or job.runner_timestamp or 0)
    states = resp.get("job_states") or []
    if not states:
        return
    last = states[-1]
    st = last.get("state")
    if st in ("done", "failed", "terminated"):
        reason_s = last.get("termination_reason") or ("done_by_runner" if st == "done" else "executor_error")
        try:
            reason = JobTerminationReason(reason_s)
        except ValueError:
            reason = JobTerminationReason.EXECUTOR_ERROR
        if "exit_status" in last:
            job.exit_status = int(last["exit_status"])
        jobs_services.terminate_job(job, reason, last.get("termination_message") or None, delay=False)
        jobs_services.mark_timing(job, "finished")
        scheduler.wake(scheduler.TERMINATING_JOBS, scheduler.RUNS)


def _record_gpu_probe(job: JobModel, doc: dict):
    """The runner ran dstack-probe (HBM/MFMA HIP kernels) before the job: keep the result as the
    instance's health so `fleet`/`instances` show it and the scheduler can avoid a bad host."""
    from dstack_amd.core.models.instances import InstanceHealth

    inst = job.instance
    try:
        health = InstanceHealth(
            healthy=bool(doc.get("healthy", True)), hbm_tb_s=doc.get("hbm_tb_s"),
            mfma_bf16_tflops=doc.get("mfma_bf16_tflops"),
            mfma_fp8_tflops=doc.get("mfma_fp8_tflops"), xgmi_gb_s=doc.get("xgmi_gb_s"),
            rccl_busbw_gb_s=doc.get("rccl_busbw_gb_s"),
            message="" if doc.get("healthy", True) else "GPU health probe below thresholds",
        )
    except Exception:  # noqa: BLE001 - a malformed probe document must not break the job
        return
    data = health.model_dump_json()
    if inst.health_data != data:
        inst.health_data = data
        inst.health_status = None if health.healthy else health.message


def _record_rccl_preflight(job: JobModel, doc: dict):
    """The runner ran the RCCL all-reduce pre-flight (DSTACK_RCCL_PREFLIGHT) before a distributed
    job: its bus bandwidth joins the instance's health, and a failed pre-flight -- or a bus bandwidth
    under ``DSTACK_RCCL_MIN_BUSBW_GB_S`` (per-link xGMI ring bound ~153 GB/s x links in use) -- marks
    the host unhealthy, so ``filter_pool_instances`` stops placing jobs on it until the shim's next
    health probe clears it.  The failing job itself already carries the probe's message.

    The floor applies to uncontended measurements only: a probe that ran CONCURRENTLY with the
    job's start-up (the runner's default, ``"mode": "concurrent"`` in its document) shares the GPUs
    and xGMI links with the job, so its bandwidth is recorded for information and never marks a
    healthy host bad; an explicit probe failure (a rank hung, a wrong sum) still does."""
    import os

    from dstack_amd.core.models.instances import InstanceHealth

    inst = job.instance
    try:
        old = InstanceHealth.model_validate_json(inst.health_data) if inst.health_data else InstanceHealth()
    except Exception:  # noqa: BLE001 - an unreadable previous document is replaced
        old = InstanceHealth()
    busbw = doc.get("rccl_busbw_gb_s")
    healthy = bool(doc.get("healthy", True))
    message = doc.get("message") or ""
    floor = os.environ.get("DSTACK_RCCL_MIN_BUSBW_GB_S")
    contended = doc.get("mode") == "concurrent"
    if healthy and floor and busbw is not None and not contended and float(busbw) < float(floor):
        healthy = False
        message = f"RCCL bus bandwidth {float(busbw):.1f} GB/s below {float(floor):.1f} GB/s"
    upd = {"rccl_busbw_gb_s": busbw if busbw is not None else old.rccl_busbw_gb_s}
    if not healthy:
        upd.update(healthy=False, message=f"RCCL pre-flight: {message or 'failed'}", source="runner")
    health = old.model_copy(update=upd)
    inst.health_data = health.model_dump_json()
    if not healthy:
        inst.health_status = health.message
        logger.warning("%s: %s", inst.name, health.message)


def _runner_unreachable(job: JobModel, err: str):
    now = get_current_datetime()
    if job.remove_at is None:
        job.remove_at = now  # first failure timestamp (reused as a marker while RUNNING)
    if now - job.remove_at > timedelta(seconds=settings.DEFAULT_RUNNER_TIMEOUT // 5):
        jobs_services.terminate_job(job, JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY,
                                    f"runner unreachable: {err}", delay=False)
        scheduler.wake(scheduler.TERMINATING_JOBS, scheduler.RUNS)
