"""Runs and jobs (reference: ``C/models/runs.py:43-510``).

A run (one configuration) expands into replicas × jobs; a job is one container on one node.
``ClusterInfo`` carries the rendezvous facts the runner turns into the DSTACK_*/RCCL env.
"""

from __future__ import annotations

import uuid
from datetime import datetime, timedelta, timezone
from enum import Enum
from typing import Any, Dict, List, Optional

from pydantic import Field, model_validator

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.common import ApplyAction, CoreModel, NetworkMode, RegistryAuth
from dstack_amd.core.models.configurations import AnyRunConfiguration
from dstack_amd.core.models.instances import (
    InstanceOfferWithAvailability,
    InstanceType,
    SSHConnectionParams,
)
from dstack_amd.core.models.profiles import (
    PROFILE_PARAM_NAMES,
    CreationPolicy,
    Profile,
    ProfileRetryPolicy,
    RetryEvent,
    SpotPolicy,
)
from dstack_amd.core.models.repos import AnyRunRepoData
from dstack_amd.core.models.resources import Memory, ResourcesSpec
from dstack_amd.core.models.unix import UnixUser
from dstack_amd.core.models.volumes import InstanceMountPoint, VolumeMountPoint


class AppSpec(CoreModel):
    port: int
    map_to_port: Optional[int] = None
    app_name: str
    url_path: Optional[str] = None
    url_query_params: Optional[Dict[str, str]] = None


class JobStatus(str, Enum):
    SUBMITTED = "submitted"
    PROVISIONING = "provisioning"
    PULLING = "pulling"
    RUNNING = "running"
    TERMINATING = "terminating"
    TERMINATED = "terminated"
    ABORTED = "aborted"
    FAILED = "failed"
    DONE = "done"

    @classmethod
    def finished_statuses(cls) -> List["JobStatus"]:
        return [cls.TERMINATED, cls.ABORTED, cls.FAILED, cls.DONE]

    def is_finished(self) -> bool:
        return self in self.finished_statuses()


class Retry(CoreModel):
    on_events: List[RetryEvent]
    duration: int

    def pretty_format(self) -> str:
        from dstack_amd.core.models.common import format_duration

        return f"{format_duration(self.duration)}[{', '.join(e.value for e in self.on_events)}]"


class RunStatus(str, Enum):
    PENDING = "pending"
    SUBMITTED = "submitted"
    PROVISIONING = "provisioning"
    RUNNING = "running"
    TERMINATING = "terminating"
    TERMINATED = "terminated"
    FAILED = "failed"
    DONE = "done"

    @classmethod
    def finished_statuses(cls) -> List["RunStatus"]:
        return [cls.TERMINATED, cls.FAILED, cls.DONE]

    def is_finished(self) -> bool:
        return self in self.finished_statuses()


class JobTerminationReason(str, Enum):
    FAILED_TO_START_DUE_TO_NO_CAPACITY = "failed_to_start_due_to_no_capacity"
    INTERRUPTED_BY_NO_CAPACITY = "interrupted_by_no_capacity"
    WAITING_INSTANCE_LIMIT_EXCEEDED = "waiting_instance_limit_exceeded"
    WAITING_RUNNER_LIMIT_EXCEEDED = "waiting_runner_limit_exceeded"
    TERMINATED_BY_USER = "terminated_by_user"
    VOLUME_ERROR = "volume_error"
    GATEWAY_ERROR = "gateway_error"
    SCALED_DOWN = "scaled_down"
    DONE_BY_RUNNER = "done_by_runner"
    ABORTED_BY_USER = "aborted_by_user"
    TERMINATED_BY_SERVER = "terminated_by_server"
    CONTAINER_EXITED_WITH_ERROR = "container_exited_with_error"
    PORTS_BINDING_FAILED = "ports_binding_failed"
    CREATING_CONTAINER_ERROR = "creating_container_error"
    EXECUTOR_ERROR = "executor_error"
    MAX_DURATION_EXCEEDED = "max_duration_exceeded"
    GPU_HEALTH_CHECK_FAILED = "gpu_health_check_failed"  # MI355X probe said the node is sick

    def to_status(self) -> JobStatus:
        return _JOB_TR_STATUS[self]

    def pretty_repr(self) -> str:
        return " ".join(self.value.split("_")).capitalize()


_JTR = JobTerminationReason
_JOB_TR_STATUS = {
    _JTR.FAILED_TO_START_DUE_TO_NO_CAPACITY: JobStatus.FAILED,
    _JTR.INTERRUPTED_BY_NO_CAPACITY: JobStatus.FAILED,
    _JTR.WAITING_INSTANCE_LIMIT_EXCEEDED: JobStatus.FAILED,
    _JTR.WAITING_RUNNER_LIMIT_EXCEEDED: JobStatus.FAILED,
    _JTR.TERMINATED_BY_USER: JobStatus.TERMINATED,
    _JTR.VOLUME_ERROR: JobStatus.FAILED,
    _JTR.GATEWAY_ERROR: JobStatus.FAILED,
    _JTR.SCALED_DOWN: JobStatus.TERMINATED,
    _JTR.DONE_BY_RUNNER: JobStatus.DONE,
    _JTR.ABORTED_BY_USER: JobStatus.ABORTED,
    _JTR.TERMINATED_BY_SERVER: JobStatus.TERMINATED,
    _JTR.CONTAINER_EXITED_WITH_ERROR: JobStatus.FAILED,
    _JTR.PORTS_BINDING_FAILED: JobStatus.FAILED,
    _JTR.CREATING_CONTAINER_ERROR: JobStatus.FAILED,
    _JTR.EXECUTOR_ERROR: JobStatus.FAILED,
    _JTR.MAX_DURATION_EXCEEDED: JobStatus.TERMINATED,
    _JTR.GPU_HEALTH_CHECK_FAILED: JobStatus.FAILED,
}


class RunTerminationReason(str, Enum):
    ALL_JOBS_DONE = "all_jobs_done"
    JOB_FAILED = "job_failed"
    RETRY_LIMIT_EXCEEDED = "retry_limit_exceeded"
    STOPPED_BY_USER = "stopped_by_user"
    ABORTED_BY_USER = "aborted_by_user"
    SERVER_ERROR = "server_error"

    def to_job_termination_reason(self) -> JobTerminationReason:
        return {
            self.ALL_JOBS_DONE: _JTR.DONE_BY_RUNNER,
            self.JOB_FAILED: _JTR.TERMINATED_BY_SERVER,
            self.RETRY_LIMIT_EXCEEDED: _JTR.TERMINATED_BY_SERVER,
            self.STOPPED_BY_USER: _JTR.TERMINATED_BY_USER,
            self.ABORTED_BY_USER: _JTR.ABORTED_BY_USER,
            self.SERVER_ERROR: _JTR.TERMINATED_BY_SERVER,
        }[self]

    def to_status(self) -> RunStatus:
        return {
            self.ALL_JOBS_DONE: RunStatus.DONE,
            self.JOB_FAILED: RunStatus.FAILED,
            self.RETRY_LIMIT_EXCEEDED: RunStatus.FAILED,
            self.STOPPED_BY_USER: RunStatus.TERMINATED,
            self.ABORTED_BY_USER: RunStatus.TERMINATED,
            self.SERVER_ERROR: RunStatus.FAILED,
        }[self]


class Requirements(CoreModel):
    resources: ResourcesSpec
    max_price: Optional[float] = None
    spot: Optional[bool] = None
    reservation: Optional[str] = None

    def pretty_format(self, resources_only: bool = False) -> str:
        res = self.resources.pretty_format()
        if not resources_only:
            if self.spot is not None:
                res += f", {'spot' if self.spot else 'on-demand'}"
            if self.max_price is not None:
                res += f" under ${self.max_price:g} per hour"
        return res


class Gateway(CoreModel):
    gateway_name: Optional[str] = None
    service_port: int
    hostname: Optional[str] = None
    public_port: int = 80
    secure: bool = False
    auth: bool = True
    options: dict = {}


class JobSpec(CoreModel):
    replica_num: int = 0
    job_num: int
    job_name: str
    jobs_per_replica: int = 1
    app_specs: Optional[List[AppSpec]] = None
    user: Optional[UnixUser] = None
    commands: List[str]
    env: Dict[str, str]
    home_dir: Optional[str] = None
    image_name: str
    privileged: bool = False
    single_branch: Optional[bool] = None
    max_duration: Optional[int] = None
    stop_duration: Optional[int] = None
    registry_auth: Optional[RegistryAuth] = None
    requirements: Requirements
    retry: Optional[Retry] = None
    volumes: Optional[List[Any]] = None
    retry_policy: ProfileRetryPolicy = Field(default_factory=lambda: ProfileRetryPolicy(retry=False))
    working_dir: Optional[str] = None
    # MI355X: run the HIP health probes before the user command (set by the configurator when the
    # job requests AMD GPUs on a fresh instance)
    gpu_probe: bool = False

    def mount_points(self):
        from dstack_amd.core.models.volumes import parse_mount_point

        return [parse_mount_point(v) for v in (self.volumes or [])]


class JobProvisioningData(CoreModel):
    backend: BackendType
    base_backend: Optional[BackendType] = None
    instance_type: InstanceType
    instance_id: str
    hostname: Optional[str] = None
    internal_ip: Optional[str] = None
    public_ip_enabled: bool = True
    instance_network: Optional[str] = None
    region: str
    availability_zone: Optional[str] = None
    reservation: Optional[str] = None
    price: float
    username: str
    ssh_port: Optional[int] = None
    dockerized: bool
    ssh_proxy: Optional[SSHConnectionParams] = None
    backend_data: Optional[str] = None

    def get_base_backend(self) -> BackendType:
        return self.base_backend or self.backend


class JobRuntimeData(CoreModel):
    network_mode: NetworkMode
    gpu: Optional[int] = None
    cpu: Optional[float] = None
    memory: Optional[Memory] = None
    ports: Optional[Dict[int, int]] = None
    volume_names: Optional[List[str]] = None
    offer: Optional[InstanceOfferWithAvailability] = None
    # MI355X: GPU indices granted on the host (xGMI-topology ordered)
    gpu_indices: Optional[List[int]] = None


class ClusterInfo(CoreModel):
    job_ips: List[str]
    master_job_ip: str
    gpus_per_job: int


class JobSubmission(CoreModel):
    id: uuid.UUID
    submission_num: int
    submitted_at: datetime
    last_processed_at: datetime
    finished_at: Optional[datetime] = None
    status: JobStatus
    termination_reason: Optional[JobTerminationReason] = None
    termination_reason_message: Optional[str] = None
    exit_status: Optional[int] = None
    job_provisioning_data: Optional[JobProvisioningData] = None
    job_runtime_data: Optional[JobRuntimeData] = None
    # cold-start instrumentation (MI355X build: event-driven scheduler timings)
    timings: Optional[Dict[str, float]] = None

    @property
    def age(self) -> timedelta:
        return datetime.now(timezone.utc) - _aware(self.submitted_at)

    @property
    def duration(self) -> timedelta:
        end = _aware(self.finished_at) if self.finished_at else datetime.now(timezone.utc)
        return end - _aware(self.submitted_at)


def _aware(dt: datetime) -> datetime:
    return dt if dt.tzinfo else dt.replace(tzinfo=timezone.utc)


class Job(CoreModel):
    job_spec: JobSpec
    job_submissions: List[JobSubmission]


class RunSpec(CoreModel):
    run_name: Optional[str] = None
    repo_id: Optional[str] = None
    repo_data: Optional[AnyRunRepoData] = None
    repo_code_hash: Optional[str] = None
    working_dir: Optional[str] = None
    configuration_path: Optional[str] = None
    configuration: AnyRunConfiguration
    profile: Optional[Profile] = None
    ssh_key_pub: str = ""

    @property
    def merged_profile(self) -> Profile:
        merged = self.profile.model_copy(deep=True) if self.profile else Profile(name="default")
        for key in PROFILE_PARAM_NAMES:
            val = getattr(self.configuration, key, None)
            if val is not None:
                setattr(merged, key, val)
        if merged.creation_policy is None:
            merged.creation_policy = CreationPolicy.REUSE_OR_CREATE
        return merged


class ServiceModelSpec(CoreModel):
    name: str
    base_url: str
    type: str


class ServiceSpec(CoreModel):
    url: str
    model: Optional[ServiceModelSpec] = None
    options: Dict[str, Any] = {}


class Run(CoreModel):
    id: uuid.UUID
    project_name: str
    user: str
    submitted_at: datetime
    last_processed_at: datetime
    status: RunStatus
    termination_reason: Optional[RunTerminationReason] = None
    run_spec: RunSpec
    jobs: List[Job]
    latest_job_submission: Optional[JobSubmission] = None
    cost: float = 0
    service: Optional[ServiceSpec] = None
    error: Optional[str] = None
    deleted: Optional[bool] = None

    @model_validator(mode="after")
    def _error(self):
        self.error = _run_error(self.termination_reason, self.jobs)
        return self


def _run_error(reason: Optional[RunTerminationReason], jobs: List[Job]) -> str:
    if reason is None:
        return ""
    if len(jobs) > 1:
        return reason.name
    jr = None
    if jobs and jobs[0].job_submissions:
        jr = jobs[0].job_submissions[-1].termination_reason
    if jr is not None and reason in (RunTerminationReason.JOB_FAILED, RunTerminationReason.SERVER_ERROR,
                                     RunTerminationReason.RETRY_LIMIT_EXCEEDED):
        return jr.name
    return reason.name


class JobPlan(CoreModel):
    job_spec: JobSpec
    offers: List[InstanceOfferWithAvailability]
    total_offers: int
    max_price: Optional[float] = None


class RunPlan(CoreModel):
    project_name: str
    user: str
    run_spec: RunSpec
    job_plans: List[JobPlan]
    current_resource: Optional[Run] = None
    action: Optional[ApplyAction] = None


class ApplyRunPlanInput(CoreModel):
    run_spec: RunSpec
    current_resource: Optional[Run] = None


class PoolInstanceOffers(CoreModel):
    pool_name: str
    instances: List[InstanceOfferWithAvailability]


def get_policy_map(spot_policy: Optional[SpotPolicy], default: SpotPolicy) -> Optional[bool]:
    spot_policy = spot_policy or default
    return {SpotPolicy.AUTO: None, SpotPolicy.SPOT: True, SpotPolicy.ONDEMAND: False}[spot_policy]
