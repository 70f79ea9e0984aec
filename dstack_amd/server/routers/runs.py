"""REST routers: runs, fleets, instances, volumes, gateways, logs, metrics (reference:
``S/routers/{runs,fleets,instances,volumes,gateways,logs,metrics,pools}.py``)."""

from __future__ import annotations

from typing import List, Optional, Tuple

from fastapi import APIRouter, Depends, Query
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.fleets import Fleet, FleetPlan, Instance
from dstack_amd.core.models.gateways import Gateway, GatewayPlan, GatewaySpec
from dstack_amd.core.models.logs import JobMetrics, JobSubmissionLogs
from dstack_amd.core.models.runs import Run, RunPlan
from dstack_amd.core.models.volumes import Volume, VolumePlan, VolumeSpec
from dstack_amd.server import schemas
from dstack_amd.server.deps import get_session
from dstack_amd.server.models import FleetModel, ProjectModel, UserModel
from dstack_amd.server.security.permissions import authenticated, project_admin, project_manager, project_member
from dstack_amd.server.services import fleets as fleets_services
from dstack_amd.server.services import gateways as gateways_services
from dstack_amd.server.services import logs as logs_services
from dstack_amd.server.services import metrics as metrics_services
from dstack_amd.server.services import pools as pools_services
from dstack_amd.server.services import projects as projects_services
from dstack_amd.server.services import runs as runs_services
from dstack_amd.server.services import volumes as volumes_services

UP = Tuple[UserModel, ProjectModel]

runs_root = APIRouter(prefix="/api/runs", tags=["runs"])
runs_router = APIRouter(prefix="/api/project/{project_name}/runs", tags=["runs"])
fleets_root = APIRouter(prefix="/api/fleets", tags=["fleets"])
fleets_router = APIRouter(prefix="/api/project/{project_name}/fleets", tags=["fleets"])
instances_root = APIRouter(prefix="/api/instances", tags=["instances"])
volumes_root = APIRouter(prefix="/api/volumes", tags=["volumes"])
volumes_router = APIRouter(prefix="/api/project/{project_name}/volumes", tags=["volumes"])
gateways_router = APIRouter(prefix="/api/project/{project_name}/gateways", tags=["gateways"])
logs_router = APIRouter(prefix="/api/project/{project_name}/logs", tags=["logs"])
metrics_router = APIRouter(prefix="/api/project/{project_name}/metrics", tags=["metrics"])
pools_root = APIRouter(prefix="/api/pools", tags=["pools"])
pool_router = APIRouter(prefix="/api/project/{project_name}/pool", tags=["pools"])
configs_router = APIRouter(prefix="/api/project/{project_name}/configurations", tags=["configurations"])


# ---- configurations ---------------------------------------------------------------------------
@configs_router.post("/parse")
def parse_configuration(body: dict, up: UP = Depends(project_member)) -> dict:
    """YAML text of a run / fleet / volume / gateway configuration -> its validated JSON form (the
    web UI's ``apply`` page has no YAML parser of its own)."""
    import yaml

    from dstack_amd.core.models.configurations import parse_apply_configuration

    try:
        data = yaml.safe_load(body.get("yaml") or "")
    except yaml.YAMLError as e:
        raise ServerClientError(f"invalid YAML: {e}")
    try:
        conf = parse_apply_configuration(data)
    except Exception as e:  # noqa: BLE001 -- validation errors go back to the form
        raise ServerClientError(str(e))
    return {"type": conf.type, "configuration": conf.model_dump(mode="json", exclude_none=True)}


# ---- runs -----------------------------------------------------------------------------------
@runs_root.post("/list")
def list_runs(body: schemas.ListRunsRequest, user: UserModel = Depends(authenticated),
              s: Session = Depends(get_session, scope="function")) -> List[Run]:
    return runs_services.list_user_runs(s, user, body.project_name, body.repo_id, body.only_active, body.limit,
                                        body.prev_submitted_at, body.ascending, body.username, body.prev_run_id)


@runs_router.post("/get")
def get_run(body: schemas.GetRunRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> Run:
    r = runs_services.get_run(s, up[1], body.run_name, body.id)
    if r is None:
        raise ResourceNotExistsError("Run not found")
    return r


@runs_router.post("/get_plan")
def get_run_plan(body: schemas.GetRunPlanRequest, up: UP = Depends(project_member),
                 s: Session = Depends(get_session, scope="function")) -> RunPlan:
    return runs_services.get_plan(s, up[1], up[0], body.run_spec, body.max_offers or 50)


@runs_router.post("/apply")
def apply_plan(body: schemas.ApplyRunPlanRequest, up: UP = Depends(project_member),
               s: Session = Depends(get_session, scope="function")) -> Run:
    return runs_services.apply_plan(s, up[1], up[0], body.plan.run_spec, body.plan.current_resource, body.force)


@runs_router.post("/submit")
def submit_run(body: schemas.SubmitRunRequest, up: UP = Depends(project_member),
               s: Session = Depends(get_session, scope="function")) -> Run:
    return runs_services.submit_run(s, up[1], up[0], body.run_spec)


@runs_router.post("/stop")
def stop_runs(body: schemas.StopRunsRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")):
    runs_services.stop_runs(s, up[1], body.runs_names, body.abort)
    return {}


@runs_router.post("/delete")
def delete_runs(body: schemas.DeleteRunsRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")):
    runs_services.delete_runs(s, up[1], body.runs_names)
    return {}


# ---- fleets ---------------------------------------------------------------------------------
@fleets_root.post("/list")
def list_all_fleets(body: Optional[schemas.ListFleetsRequest] = None, user: UserModel = Depends(authenticated),
                    s: Session = Depends(get_session, scope="function")) -> List[Fleet]:
    out = []
    for p in projects_services.list_user_projects(s, user):
        if body and body.project_name and p.name != body.project_name:
            continue
        out += [fleets_services.fleet_model_to_fleet(f) for f in fleets_services.list_project_fleets(s, p)]
    return out


@fleets_router.post("/list")
def list_fleets(up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> List[Fleet]:
    return [fleets_services.fleet_model_to_fleet(f) for f in fleets_services.list_project_fleets(s, up[1])]


@fleets_router.post("/get")
def get_fleet(body: schemas.GetFleetRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> Fleet:
    if body.id is not None:  # by id: deleted fleets too (reference routers/fleets.py get)
        f = s.get(FleetModel, body.id)
        f = f if f is not None and f.project_id == up[1].id else None
    else:
        f = fleets_services.get_fleet_by_name(s, up[1], body.name) if body.name else None
    if f is None:
        raise ResourceNotExistsError("Fleet not found")
    return fleets_services.fleet_model_to_fleet(f)


@fleets_router.post("/get_plan")
def get_fleet_plan(body: schemas.GetFleetPlanRequest, up: UP = Depends(project_member),
                   s: Session = Depends(get_session, scope="function")) -> FleetPlan:
    return fleets_services.get_plan(s, up[1], up[0], body.spec)


@fleets_router.post("/create")
def create_fleet(body: schemas.CreateFleetRequest, up: UP = Depends(project_manager),
                 s: Session = Depends(get_session, scope="function")) -> Fleet:
    return fleets_services.create_fleet(s, up[1], up[0], body.spec)


@fleets_router.post("/delete")
def delete_fleets(body: schemas.DeleteFleetsRequest, up: UP = Depends(project_manager),
                  s: Session = Depends(get_session, scope="function")):
    fleets_services.delete_fleets(s, up[1], body.names, up[0])
    return {}


@fleets_router.post("/delete_instances")
def delete_fleet_instances(body: schemas.DeleteFleetInstancesRequest, up: UP = Depends(project_manager),
                           s: Session = Depends(get_session, scope="function")):
    fleets_services.delete_fleet_instances(s, up[1], body.name, body.instance_nums, up[0])
    return {}


# ---- instances / legacy pools ---------------------------------------------------------------
@instances_root.post("/list")
def list_instances(body: Optional[schemas.ListInstancesRequest] = None, user: UserModel = Depends(authenticated),
                   s: Session = Depends(get_session, scope="function")) -> List[Instance]:
    body = body or schemas.ListInstancesRequest()
    rows = []
    for p in projects_services.list_user_projects(s, user):
        if body.project_names and p.name not in body.project_names:
            continue
        if body.project_name and p.name != body.project_name:
            continue
        for inst in pools_services.list_project_instances(s, p, include_terminated=not body.only_active):
            if body.fleet_ids and inst.fleet_id not in body.fleet_ids:
                continue
            if body.pool_name and (inst.pool is None or inst.pool.name != body.pool_name):
                continue
            rows.append(inst)
    # keyset pagination (reference routers/instances.py): order by (created_at, id), newest first
    rows.sort(key=lambda i: (i.created_at, str(i.id)), reverse=not body.ascending)
    if body.prev_created_at is not None:
        key = (body.prev_created_at.replace(tzinfo=None), str(body.prev_id or ""))
        rows = [i for i in rows if ((i.created_at, str(i.id)) > key if body.ascending else (i.created_at, str(i.id)) < key)]
    return [pools_services.instance_model_to_instance(i) for i in rows[: body.limit]]


@pools_root.post("/list_instances")
def pools_list_instances(body: Optional[schemas.ListInstancesRequest] = None, user: UserModel = Depends(authenticated),
                         s: Session = Depends(get_session, scope="function")) -> List[Instance]:
    return list_instances(body, user, s)


@pool_router.post("/list")
def pool_list(up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")):
    return pools_services.list_project_pools(s, up[1])


@pool_router.post("/show")
def pool_show(body: Optional[schemas.ShowPoolRequest] = None, up: UP = Depends(project_member),
              s: Session = Depends(get_session, scope="function")):
    return pools_services.show_pool_instances(s, up[1], body.name if body else None)


@pool_router.post("/create")
def pool_create(body: schemas.CreatePoolRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")):
    pools_services.create_pool(s, up[1], body.name)
    return None


@pool_router.post("/set_default")
def pool_set_default(body: schemas.SetDefaultPoolRequest, up: UP = Depends(project_member),
                     s: Session = Depends(get_session, scope="function")):
    pools_services.set_default_pool(s, up[1], body.pool_name)
    return None


@pool_router.post("/delete")
def pool_delete(body: schemas.DeletePoolRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")):
    pools_services.delete_pool(s, up[1], body.name)
    return None


@pool_router.post("/remove")
def pool_remove_instance(body: schemas.RemoveInstanceRequest, up: UP = Depends(project_member),
                         s: Session = Depends(get_session, scope="function")):
    from dstack_amd.server.services.permissions import check_can_manage_ssh_fleets

    pool = pools_services.get_pool(s, up[1], body.pool_name)
    if pool is not None and any(i.name == body.instance_name and i.backend == "remote" and not i.deleted
                                for i in pool.instances):
        check_can_manage_ssh_fleets(up[0], up[1])  # SSH hosts: same rule as SSH fleets
    pools_services.remove_instance(s, up[1], body.pool_name, body.instance_name, body.force)
    return None


@pool_router.post("/add_remote")
def pool_add_remote(body: schemas.AddRemoteInstanceRequest, up: UP = Depends(project_member),
                    s: Session = Depends(get_session, scope="function")) -> Instance:
    from dstack_amd.server.services.permissions import check_can_manage_ssh_fleets

    check_can_manage_ssh_fleets(up[0], up[1])  # an SSH host is an SSH fleet by another door
    if not body.host.strip() or not body.ssh_user.strip() or not body.ssh_keys:
        raise ServerClientError("Host, user or ssh keys are empty")
    return pools_services.add_remote(s, up[1], body.pool_name, body.instance_name, body.instance_network,
                                     body.region, body.host, body.port or 22, body.ssh_user, body.ssh_keys)


# legacy: get_offers / create_instance live under runs in the reference (routers/runs.py:183-219)
@runs_router.post("/get_offers")
def runs_get_offers(body: schemas.GetOffersRequest, up: UP = Depends(project_member),
                    s: Session = Depends(get_session, scope="function")):
    from dstack_amd.core.models.runs import PoolInstanceOffers
    from dstack_amd.server.services import offers as offers_services

    pool = pools_services.get_or_create_pool_by_name(s, up[1], body.profile.pool_name)
    offers = offers_services.get_offers_by_requirements(s, up[1], body.profile, body.requirements)
    return PoolInstanceOffers(pool_name=pool.name, instances=[o for _, o in offers])


@runs_router.post("/create_instance")
def runs_create_instance(body: schemas.CreateInstanceRequest, up: UP = Depends(project_member),
                         s: Session = Depends(get_session, scope="function")) -> Instance:
    return fleets_services.create_instance(s, up[1], up[0], body.profile, body.requirements)


# ---- volumes --------------------------------------------------------------------------------
@volumes_root.post("/list")
def list_all_volumes(body: Optional[schemas.ListVolumesRequest] = None, user: UserModel = Depends(authenticated),
                     s: Session = Depends(get_session, scope="function")) -> List[Volume]:
    out = []
    for p in projects_services.list_user_projects(s, user):
        if body and body.project_name and p.name != body.project_name:
            continue
        out += [volumes_services.volume_model_to_volume(v) for v in volumes_services.list_project_volumes(s, p)]
    return out


@volumes_router.post("/list")
def list_volumes(up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> List[Volume]:
    return [volumes_services.volume_model_to_volume(v) for v in volumes_services.list_project_volumes(s, up[1])]


@volumes_router.post("/get")
def get_volume(body: schemas.GetVolumeRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> Volume:
    v = volumes_services.get_volume_by_name(s, up[1], body.name)
    if v is None:
        raise ResourceNotExistsError("Volume not found")
    return volumes_services.volume_model_to_volume(v)


@volumes_router.post("/get_plan")
def get_volume_plan(body: dict, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> VolumePlan:
    return volumes_services.get_plan(s, up[1], up[0], VolumeSpec.model_validate(body["spec"]))


@volumes_router.post("/create")
def create_volume(body: schemas.CreateVolumeRequest, up: UP = Depends(project_member),
                  s: Session = Depends(get_session, scope="function")) -> Volume:
    return volumes_services.create_volume(s, up[1], up[0], body.configuration)


@volumes_router.post("/delete")
def delete_volumes(body: schemas.DeleteVolumesRequest, up: UP = Depends(project_member),
                   s: Session = Depends(get_session, scope="function")):
    volumes_services.delete_volumes(s, up[1], body.names)
    return {}


# ---- gateways -------------------------------------------------------------------------------
@gateways_router.post("/list")
def list_gateways(up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> List[Gateway]:
    return [gateways_services.gateway_model_to_gateway(g) for g in gateways_services.list_project_gateways(s, up[1])]


@gateways_router.post("/get")
def get_gateway(body: schemas.GetGatewayRequest, up: UP = Depends(project_member),
                s: Session = Depends(get_session, scope="function")) -> Gateway:
    g = gateways_services.get_gateway_by_name(s, up[1], body.name)
    if g is None:
        raise ResourceNotExistsError("Gateway not found")
    return gateways_services.gateway_model_to_gateway(g)


@gateways_router.post("/get_plan")
def get_gateway_plan(body: dict, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> GatewayPlan:
    return gateways_services.get_plan(s, up[1], up[0], GatewaySpec.model_validate(body["spec"]))


@gateways_router.post("/create")
def create_gateway(body: schemas.CreateGatewayRequest, up: UP = Depends(project_admin),
                   s: Session = Depends(get_session, scope="function")) -> Gateway:
    return gateways_services.create_gateway(s, up[1], body.configuration)


@gateways_router.post("/delete")
def delete_gateways(body: schemas.DeleteGatewaysRequest, up: UP = Depends(project_admin),
                    s: Session = Depends(get_session, scope="function")):
    gateways_services.delete_gateways(s, up[1], body.names)
    return {}


@gateways_router.post("/set_default")
def set_default_gateway(body: schemas.SetDefaultGatewayRequest, up: UP = Depends(project_admin),
                        s: Session = Depends(get_session, scope="function")):
    gateways_services.set_default_gateway(s, up[1], body.name)
    return {}


@gateways_router.post("/set_wildcard_domain")
def set_wildcard_domain(body: schemas.SetWildcardDomainRequest, up: UP = Depends(project_admin),
                        s: Session = Depends(get_session, scope="function")) -> Gateway:
    return gateways_services.set_wildcard_domain(s, up[1], body.name, body.wildcard_domain)


# ---- logs / metrics -------------------------------------------------------------------------
@logs_router.post("/poll")
def poll_logs(body: schemas.PollLogsRequest, up: UP = Depends(project_member)) -> JobSubmissionLogs:
    from datetime import datetime

    start, end = body.start_time, body.end_time
    if body.next_token:
        try:
            token = datetime.fromisoformat(body.next_token)
        except ValueError:
            raise ServerClientError("invalid next_token")
        # the token is the last returned event's timestamp: the next page continues past it in the
        # direction of the listing
        if body.descending:
            end = token
        else:
            start = token
    return logs_services.get_default_log_storage().poll_logs(
        up[1].name, body.run_name, str(body.job_submission_id), start, end, body.descending, body.limit,
        body.diagnose)


@metrics_router.get("/job/{run_name}")
def get_job_metrics(run_name: str, replica_num: int = Query(0), job_num: int = Query(0), limit: int = Query(2),
                    up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> JobMetrics:
    run = runs_services.get_run_by_name_or_error(s, up[1], run_name)
    jobs = [j for j in run.jobs if j.replica_num == replica_num and j.job_num == job_num]
    if not jobs:
        raise ResourceNotExistsError("Job not found")
    job = max(jobs, key=lambda j: j.submission_num)
    return metrics_services.get_job_metrics(s, job, limit)
