"""ORM schema (reference: ``S/models.py:148-651``).

JSON-serialised pydantic payloads live in TEXT columns (``*_data``); sensitive columns use
``EncryptedString`` (AES-GCM, ``services/encryption.py``).  All datetimes are naive UTC.
"""

from __future__ import annotations

import uuid
from datetime import datetime, timezone
from typing import List, Optional

from sqlalchemy import (
    BigInteger,
    Boolean,
    Column,
    DateTime,
    Float,
    ForeignKey,
    Index,
    Integer,
    LargeBinary,
    String,
    Table,
    Text,
    TypeDecorator,
    UniqueConstraint,
)
from sqlalchemy.orm import DeclarativeBase, Mapped, mapped_column, relationship

from dstack_amd.server.services import encryption


def utcnow() -> datetime:
    return datetime.now(timezone.utc).replace(tzinfo=None)


class EncryptedString(TypeDecorator):
    impl = Text
    cache_ok = True

    def process_bind_param(self, value, dialect):
        if value is None:
            return None
        return encryption.encrypt(value)

    def process_result_value(self, value, dialect):
        if value is None:
            return None
        return encryption.decrypt(value)


class UUIDStr(TypeDecorator):
    impl = String(36)
    cache_ok = True

    def process_bind_param(self, value, dialect):
        return None if value is None else str(value)

    def process_result_value(self, value, dialect):
        return None if value is None else uuid.UUID(value)


class Base(DeclarativeBase):
    pass


def _id():
    return mapped_column(UUIDStr, primary_key=True, default=uuid.uuid4)


class UserModel(Base):
    __tablename__ = "users"
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(50), unique=True)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    token: Mapped[str] = mapped_column(EncryptedString)
    token_hash: Mapped[str] = mapped_column(String(128), unique=True)
    global_role: Mapped[str] = mapped_column(String(20))
    email: Mapped[Optional[str]] = mapped_column(String(200), nullable=True)
    active: Mapped[bool] = mapped_column(Boolean, default=True)
    projects_quota: Mapped[int] = mapped_column(Integer, default=3)


class ProjectModel(Base):
    __tablename__ = "projects"
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(50), unique=True)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    owner_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("users.id", ondelete="CASCADE"))
    owner: Mapped[UserModel] = relationship(lazy="joined")
    members: Mapped[List["MemberModel"]] = relationship(back_populates="project", lazy="selectin",
                                                        order_by="MemberModel.member_num")
    backends: Mapped[List["BackendModel"]] = relationship(back_populates="project", lazy="selectin")
    ssh_private_key: Mapped[str] = mapped_column(Text)
    ssh_public_key: Mapped[str] = mapped_column(Text)
    default_gateway_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, nullable=True)
    default_pool_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, nullable=True)


class MemberModel(Base):
    __tablename__ = "members"
    id: Mapped[uuid.UUID] = _id()
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship(back_populates="members")
    user_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("users.id", ondelete="CASCADE"))
    user: Mapped[UserModel] = relationship(lazy="joined")
    project_role: Mapped[str] = mapped_column(String(20))
    member_num: Mapped[Optional[int]] = mapped_column(Integer, nullable=True)


class BackendModel(Base):
    __tablename__ = "backends"
    __table_args__ = (UniqueConstraint("project_id", "type"),)
    id: Mapped[uuid.UUID] = _id()
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship(back_populates="backends")
    type: Mapped[str] = mapped_column(String(30))
    config: Mapped[str] = mapped_column(Text)
    auth: Mapped[str] = mapped_column(EncryptedString)


class RepoModel(Base):
    __tablename__ = "repos"
    __table_args__ = (UniqueConstraint("project_id", "name"),)
    id: Mapped[uuid.UUID] = _id()
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    name: Mapped[str] = mapped_column(String(100))
    type: Mapped[str] = mapped_column(String(20))
    info: Mapped[str] = mapped_column(Text)
    creds: Mapped[Optional[str]] = mapped_column(EncryptedString, nullable=True)


class RepoCredsModel(Base):
    __tablename__ = "repo_creds"
    __table_args__ = (UniqueConstraint("repo_id", "user_id"),)
    id: Mapped[uuid.UUID] = _id()
    repo_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("repos.id", ondelete="CASCADE"))
    user_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("users.id", ondelete="CASCADE"))
    creds: Mapped[str] = mapped_column(EncryptedString)


class CodeModel(Base):
    __tablename__ = "codes"
    __table_args__ = (UniqueConstraint("repo_id", "blob_hash"),)
    id: Mapped[uuid.UUID] = _id()
    repo_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("repos.id", ondelete="CASCADE"))
    blob_hash: Mapped[str] = mapped_column(String(128))
    blob: Mapped[Optional[bytes]] = mapped_column(LargeBinary, nullable=True)  # None -> stored in S3


class FleetModel(Base):
    __tablename__ = "fleets"
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(100))
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    last_processed_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    deleted_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    status: Mapped[str] = mapped_column(String(20))
    status_message: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    spec: Mapped[str] = mapped_column(Text)
    instances: Mapped[List["InstanceModel"]] = relationship(back_populates="fleet", lazy="selectin")
    runs: Mapped[List["RunModel"]] = relationship(back_populates="fleet")


class PoolModel(Base):
    __tablename__ = "pools"
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(50))
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    deleted_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    instances: Mapped[List["InstanceModel"]] = relationship(back_populates="pool")


volumes_attachments = Table(
    "volumes_attachments",
    Base.metadata,
    Column("volume_id", UUIDStr, ForeignKey("volumes.id", ondelete="CASCADE"), primary_key=True),
    Column("instance_id", UUIDStr, ForeignKey("instances.id", ondelete="CASCADE"), primary_key=True),
    Column("attachment_data", Text, nullable=True),
)


class InstanceModel(Base):
    __tablename__ = "instances"
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(100))
    instance_num: Mapped[int] = mapped_column(Integer, default=0)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    last_processed_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    deleted_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    pool_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, ForeignKey("pools.id"), nullable=True)
    pool: Mapped[Optional[PoolModel]] = relationship(back_populates="instances")
    fleet_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, ForeignKey("fleets.id"), nullable=True)
    fleet: Mapped[Optional[FleetModel]] = relationship(back_populates="instances")
    status: Mapped[str] = mapped_column(String(20))
    unreachable: Mapped[bool] = mapped_column(Boolean, default=False)
    started_at: Mapped[Optional[datetime]] = mapped_column(DateTime, default=utcnow, nullable=True)
    finished_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    profile: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    requirements: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    instance_configuration: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    termination_policy: Mapped[Optional[str]] = mapped_column(String(50), nullable=True)
    termination_idle_time: Mapped[int] = mapped_column(Integer, default=300)
    retry_policy: Mapped[bool] = mapped_column(Boolean, default=False)
    retry_policy_duration: Mapped[Optional[int]] = mapped_column(Integer, nullable=True)
    last_retry_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    termination_deadline: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    termination_reason: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    health_status: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    health_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)  # InstanceHealth json
    first_termination_retry_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    last_termination_retry_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    backend: Mapped[Optional[str]] = mapped_column(String(30), nullable=True)
    backend_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    offer: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    region: Mapped[Optional[str]] = mapped_column(String(200), nullable=True)
    price: Mapped[Optional[float]] = mapped_column(Float, nullable=True)
    job_provisioning_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    remote_connection_info: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    host_topology: Mapped[Optional[str]] = mapped_column(Text, nullable=True)  # HostTopology json
    total_blocks: Mapped[Optional[int]] = mapped_column(Integer, nullable=True)
    busy_blocks: Mapped[int] = mapped_column(Integer, default=0)
    # bitmask of GPU indices currently granted to jobs (xGMI-aware allocation)
    busy_gpus: Mapped[str] = mapped_column(Text, default="")
    jobs: Mapped[List["JobModel"]] = relationship(back_populates="instance")
    last_job_processed_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    volumes: Mapped[List["VolumeModel"]] = relationship(secondary=volumes_attachments, back_populates="instances")
    # SSH-fleet deploy lease: the server replica running this host's deploy and when it started;
    # other replicas leave the instance alone until the lease expires (process_instances._add_remote)
    deploy_owner: Mapped[Optional[str]] = mapped_column(String(100), nullable=True)
    deploy_started_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)


class RunModel(Base):
    __tablename__ = "runs"
    id: Mapped[uuid.UUID] = _id()
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    user_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("users.id", ondelete="CASCADE"))
    user: Mapped[UserModel] = relationship()
    repo_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("repos.id", ondelete="CASCADE"))
    repo: Mapped[RepoModel] = relationship()
    fleet_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, ForeignKey("fleets.id"), nullable=True)
    fleet: Mapped[Optional[FleetModel]] = relationship(back_populates="runs")
    run_name: Mapped[str] = mapped_column(String(100))
    submitted_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    last_processed_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    status: Mapped[str] = mapped_column(String(20))
    termination_reason: Mapped[Optional[str]] = mapped_column(String(50), nullable=True)
    resubmission_attempt: Mapped[int] = mapped_column(Integer, default=0)
    run_spec: Mapped[str] = mapped_column(Text)
    service_spec: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    desired_replica_count: Mapped[int] = mapped_column(Integer, default=1)
    gateway_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, ForeignKey("gateways.id"), nullable=True)
    gateway: Mapped[Optional["GatewayModel"]] = relationship()
    jobs: Mapped[List["JobModel"]] = relationship(back_populates="run", lazy="selectin",
                                                  order_by="(JobModel.replica_num, JobModel.job_num, "
                                                           "JobModel.submission_num)")


class JobModel(Base):
    __tablename__ = "jobs"
    id: Mapped[uuid.UUID] = _id()
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    run_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("runs.id", ondelete="CASCADE"))
    run: Mapped[RunModel] = relationship(back_populates="jobs")
    run_name: Mapped[str] = mapped_column(String(100))
    job_num: Mapped[int] = mapped_column(Integer)
    job_name: Mapped[str] = mapped_column(String(100))
    replica_num: Mapped[int] = mapped_column(Integer, default=0)
    submission_num: Mapped[int] = mapped_column(Integer)
    submitted_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    last_processed_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    finished_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    status: Mapped[str] = mapped_column(String(20))
    termination_reason: Mapped[Optional[str]] = mapped_column(String(50), nullable=True)
    termination_reason_message: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    exit_status: Mapped[Optional[int]] = mapped_column(Integer, nullable=True)
    job_spec_data: Mapped[str] = mapped_column(Text)
    job_provisioning_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    job_runtime_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    runner_timestamp: Mapped[Optional[int]] = mapped_column(BigInteger, nullable=True)
    remove_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    volumes_detached_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    instance_assigned: Mapped[bool] = mapped_column(Boolean, default=False)
    instance_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, ForeignKey("instances.id"), nullable=True)
    instance: Mapped[Optional[InstanceModel]] = relationship(back_populates="jobs")
    used_instance_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, nullable=True)
    timings: Mapped[Optional[str]] = mapped_column(Text, nullable=True)  # cold-start stage timestamps json


class GatewayModel(Base):
    __tablename__ = "gateways"
    __table_args__ = (UniqueConstraint("project_id", "name"),)
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(100))
    region: Mapped[str] = mapped_column(String(100))
    wildcard_domain: Mapped[Optional[str]] = mapped_column(String(200), nullable=True)
    configuration: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    status: Mapped[str] = mapped_column(String(20))
    status_message: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    last_processed_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    backend_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("backends.id", ondelete="CASCADE"))
    backend: Mapped[BackendModel] = relationship(lazy="joined")
    gateway_compute_id: Mapped[Optional[uuid.UUID]] = mapped_column(
        UUIDStr, ForeignKey("gateway_computes.id", ondelete="CASCADE"), nullable=True
    )
    gateway_compute: Mapped[Optional["GatewayComputeModel"]] = relationship(lazy="joined")


class GatewayComputeModel(Base):
    __tablename__ = "gateway_computes"
    id: Mapped[uuid.UUID] = _id()
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    instance_id: Mapped[str] = mapped_column(String(100))
    ip_address: Mapped[str] = mapped_column(String(100))
    hostname: Mapped[Optional[str]] = mapped_column(String(200), nullable=True)
    configuration: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    backend_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    region: Mapped[str] = mapped_column(String(100))
    backend_id: Mapped[Optional[uuid.UUID]] = mapped_column(UUIDStr, ForeignKey("backends.id", ondelete="CASCADE"),
                                                            nullable=True)
    ssh_private_key: Mapped[str] = mapped_column(Text)
    ssh_public_key: Mapped[str] = mapped_column(Text)
    active: Mapped[bool] = mapped_column(Boolean, default=True)
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    app_updated_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)


class VolumeModel(Base):
    __tablename__ = "volumes"
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(100))
    user_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("users.id", ondelete="CASCADE"))
    user: Mapped[UserModel] = relationship()
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    last_processed_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    deleted_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    status: Mapped[str] = mapped_column(String(20))
    status_message: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    configuration: Mapped[str] = mapped_column(Text)
    volume_provisioning_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    volume_attachment_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    instances: Mapped[List[InstanceModel]] = relationship(secondary=volumes_attachments, back_populates="volumes")


class PlacementGroupModel(Base):
    __tablename__ = "placement_groups"
    id: Mapped[uuid.UUID] = _id()
    name: Mapped[str] = mapped_column(String(100))
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    project: Mapped[ProjectModel] = relationship()
    fleet_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("fleets.id"))
    fleet: Mapped[FleetModel] = relationship()
    fleet_deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    last_processed_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    deleted: Mapped[bool] = mapped_column(Boolean, default=False)
    deleted_at: Mapped[Optional[datetime]] = mapped_column(DateTime, nullable=True)
    configuration: Mapped[str] = mapped_column(Text)
    provisioning_data: Mapped[Optional[str]] = mapped_column(Text, nullable=True)


class JobMetricsPoint(Base):
    __tablename__ = "job_metrics_points"
    # the newest samples of a job (gpu_util autoscaler, `dstack stats`); migration 6 for older DBs
    __table_args__ = (Index("ix_job_metrics_points_job_ts", "job_id", "timestamp_micro"),)
    id: Mapped[uuid.UUID] = _id()
    job_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("jobs.id", ondelete="CASCADE"), index=True)
    timestamp_micro: Mapped[int] = mapped_column(BigInteger)
    cpu_usage_micro: Mapped[int] = mapped_column(BigInteger)
    memory_usage_bytes: Mapped[int] = mapped_column(BigInteger)
    memory_working_set_bytes: Mapped[int] = mapped_column(BigInteger)
    gpus_memory_usage_bytes: Mapped[str] = mapped_column(Text)  # json list
    gpus_util_percent: Mapped[str] = mapped_column(Text)  # json list
    gpus_power_watts: Mapped[Optional[str]] = mapped_column(Text, nullable=True)  # json list (amdsmi)
    gpus_temperature_c: Mapped[Optional[str]] = mapped_column(Text, nullable=True)
    # json list of per-GPU dicts: HBM controller activity and xGMI link state / accumulated KiB
    gpus_extra: Mapped[Optional[str]] = mapped_column(Text, nullable=True)


class SecretModel(Base):
    __tablename__ = "secrets"
    __table_args__ = (UniqueConstraint("project_id", "name"),)
    id: Mapped[uuid.UUID] = _id()
    project_id: Mapped[uuid.UUID] = mapped_column(UUIDStr, ForeignKey("projects.id", ondelete="CASCADE"))
    created_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
    name: Mapped[str] = mapped_column(String(200))
    value: Mapped[str] = mapped_column(EncryptedString)


class SchemaVersionModel(Base):
    __tablename__ = "schema_version"
    version: Mapped[int] = mapped_column(Integer, primary_key=True)
    applied_at: Mapped[datetime] = mapped_column(DateTime, default=utcnow)
