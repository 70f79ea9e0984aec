"""Request bodies of the REST API (reference: ``S/schemas/*.py``)."""

from __future__ import annotations

from datetime import datetime
from typing import Any, Dict, List, Optional
from uuid import UUID

from pydantic import ConfigDict

from dstack_amd.core.models.common import CoreModel
from dstack_amd.core.models.fleets import FleetSpec
from dstack_amd.core.models.gateways import GatewayConfiguration
from dstack_amd.core.models.instances import SSHKey
from dstack_amd.core.models.profiles import Profile
from dstack_amd.core.models.runs import ApplyRunPlanInput, Requirements, RunSpec
from dstack_amd.core.models.users import GlobalRole, ProjectRole
from dstack_amd.core.models.volumes import VolumeConfiguration


class _Req(CoreModel):
    model_config = ConfigDict(extra="ignore")


# users
class GetUserRequest(_Req):
    username: str


class CreateUserRequest(_Req):
    username: str
    global_role: GlobalRole = GlobalRole.USER
    email: Optional[str] = None
    active: bool = True


class UpdateUserRequest(CreateUserRequest):
    pass


class RefreshTokenRequest(_Req):
    username: str


class DeleteUsersRequest(_Req):
    users: List[str]


# projects
class CreateProjectRequest(_Req):
    project_name: str


class DeleteProjectsRequest(_Req):
    projects_names: List[str]


class MemberSetting(_Req):
    username: str
    project_role: ProjectRole


class SetProjectMembersRequest(_Req):
    members: List[MemberSetting]


# backends
class CreateBackendYAMLRequest(_Req):
    config_yaml: str


class DeleteBackendsRequest(_Req):
    backends_names: List[str]


# fleets
class GetFleetRequest(_Req):
    name: Optional[str] = None
    id: Optional[UUID] = None


class GetFleetPlanRequest(_Req):
    spec: FleetSpec


class CreateFleetRequest(_Req):
    spec: FleetSpec


class DeleteFleetsRequest(_Req):
    names: List[str]


class DeleteFleetInstancesRequest(_Req):
    name: str
    instance_nums: List[int]


class ListFleetsRequest(_Req):
    project_name: Optional[str] = None
    only_active: bool = False


class ListInstancesRequest(_Req):
    project_names: Optional[List[str]] = None
    fleet_ids: Optional[List[UUID]] = None
    pool_name: Optional[str] = None
    project_name: Optional[str] = None
    only_active: bool = False
    # keyset pagination over (created, id), newest first unless ascending
    prev_created_at: Optional[datetime] = None
    prev_id: Optional[UUID] = None
    ascending: bool = False
    limit: int = 1000


# repos
class GetRepoRequest(_Req):
    repo_id: str
    include_creds: bool = False


class InitRepoRequest(_Req):
    repo_id: str
    repo_info: Dict[str, Any]
    repo_creds: Optional[Dict[str, Any]] = None


class DeleteReposRequest(_Req):
    repos_ids: List[str]


# runs
class ListRunsRequest(_Req):
    project_name: Optional[str] = None
    repo_id: Optional[str] = None
    username: Optional[str] = None
    only_active: bool = False
    prev_submitted_at: Optional[datetime] = None
    prev_run_id: Optional[UUID] = None
    limit: int = 100
    ascending: bool = False


class GetRunRequest(_Req):
    run_name: Optional[str] = None
    id: Optional[UUID] = None


class GetRunPlanRequest(_Req):
    run_spec: RunSpec
    max_offers: Optional[int] = None


class SubmitRunRequest(_Req):
    run_spec: RunSpec


class ApplyRunPlanRequest(_Req):
    plan: ApplyRunPlanInput
    force: bool = False


class StopRunsRequest(_Req):
    runs_names: List[str]
    abort: bool = False


class DeleteRunsRequest(_Req):
    runs_names: List[str]


# logs / secrets / gateways / volumes
class PollLogsRequest(_Req):
    run_name: str
    job_submission_id: UUID
    start_time: Optional[datetime] = None
    end_time: Optional[datetime] = None
    descending: bool = False
    limit: int = 1000
    diagnose: bool = False
    next_token: Optional[str] = None


class GetSecretRequest(_Req):
    name: str


class AddSecretRequest(_Req):
    name: str
    value: str


class DeleteSecretsRequest(_Req):
    secrets_names: List[str]


class GetGatewayRequest(_Req):
    name: str


class CreateGatewayRequest(_Req):
    configuration: GatewayConfiguration


class DeleteGatewaysRequest(_Req):
    names: List[str]


class SetDefaultGatewayRequest(_Req):
    name: str


class SetWildcardDomainRequest(_Req):
    name: str
    wildcard_domain: Optional[str] = None


class GetVolumeRequest(_Req):
    name: str


class CreateVolumeRequest(_Req):
    configuration: VolumeConfiguration


class DeleteVolumesRequest(_Req):
    names: List[str]


class ListVolumesRequest(_Req):
    project_name: Optional[str] = None
    only_active: bool = False




# ---- legacy pools (reference: S/schemas/pools.py, S/schemas/runs.py AddRemoteInstanceRequest) ----
class CreatePoolRequest(_Req):
    name: str


class SetDefaultPoolRequest(_Req):
    pool_name: str


class DeletePoolRequest(_Req):
    name: str
    force: bool = False


class ShowPoolRequest(_Req):
    name: Optional[str] = None


class RemoveInstanceRequest(_Req):
    pool_name: str
    instance_name: str
    force: bool = False


class AddRemoteInstanceRequest(_Req):
    pool_name: Optional[str] = None
    instance_name: Optional[str] = None
    instance_network: Optional[str] = None
    region: Optional[str] = None
    host: str
    port: Optional[int] = None
    ssh_user: str
    ssh_keys: List[SSHKey]


class GetOffersRequest(_Req):
    profile: Profile
    requirements: Requirements


class CreateInstanceRequest(_Req):
    profile: Profile
    requirements: Requirements
