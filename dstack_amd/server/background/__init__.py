"""Reconciler registration (reference: ``S/background/__init__.py:34-87``).

Intervals keep the reference's fallback cadence (jobs/instances 4 s ± 2, runs 2 s ± 1, metrics
10 s, fleets 10 s, volumes/gateways 10 s, placement groups 30 s) except RUNNING-job log pulls,
which poll every 1 s (loopback/pooled-tunnel HTTP is cheap) so logs reach the CLI sooner; all
stage transitions are event-driven through ``scheduler.wake``.
"""

from __future__ import annotations

import logging

from sqlalchemy import select

from dstack_amd.core.models.gateways import GatewayStatus
from dstack_amd.server import settings
from dstack_amd.server.background import scheduler as sch
from dstack_amd.server.background.tasks.process_fleets import process_fleets
from dstack_amd.server.background.tasks.process_instances import process_instances
from dstack_amd.server.background.tasks.process_metrics import collect_metrics, delete_metrics
from dstack_amd.server.background.tasks.process_placement_groups import process_placement_groups
from dstack_amd.server.background.tasks.process_running_jobs import process_running_jobs
from dstack_amd.server.background.tasks.process_runs import process_runs
from dstack_amd.server.background.tasks.process_submitted_jobs import process_submitted_jobs
from dstack_amd.server.background.tasks.process_terminating_jobs import process_terminating_jobs
from dstack_amd.server.background.tasks.process_volumes import process_submitted_volumes
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import GatewayModel

logger = logging.getLogger(__name__)


def process_submitted_gateways() -> bool:
    """SUBMITTED gateways get their compute (``provision_gateway``); PROVISIONING ones are connected
    (``connect_gateway``: RUNNING once the control API answers, FAILED after the deadline)."""
    from dstack_amd.server.services.gateways import connect_gateway, provision_gateway

    with session_scope() as s:
        for g in s.execute(select(GatewayModel).where(GatewayModel.status == GatewayStatus.SUBMITTED.value)).scalars():
            provision_gateway(s, g)
    with session_scope() as s:
        for g in s.execute(select(GatewayModel).where(GatewayModel.status == GatewayStatus.PROVISIONING.value)).scalars():
            connect_gateway(s, g)
    return False


def process_gateways_connections() -> bool:
    """Collect RPS stats from running gateways for the autoscaler (reference:
    ``process_gateways.py:25-93``)."""
    from dstack_amd.server.services.gateways import gateway_stats
    from dstack_amd.server.services.services import get_request_stats

    from dstack_amd.server.models import RunModel

    with session_scope() as s:
        for g in s.execute(select(GatewayModel).where(GatewayModel.status == GatewayStatus.RUNNING.value)).scalars():
            if g.gateway_compute is None:
                continue
            try:
                stats = gateway_stats(g)
            except Exception as e:  # noqa: BLE001
                logger.debug("gateway %s stats: %s", g.name, e)
                continue
            for item in stats if isinstance(stats, list) else []:
                run = s.execute(select(RunModel).where(RunModel.project_id == g.project_id,
                                                       RunModel.run_name == item.get("run_name"),
                                                       RunModel.deleted == False)  # noqa: E712
                                .order_by(RunModel.submitted_at.desc())).scalars().first()
                w = (item.get("stats") or {}).get("60")
                if run is not None and w is not None:
                    get_request_stats().set_external(run.id, w["requests"] / 60.0, w["request_time"])
    return False


def start_background_tasks() -> sch.Scheduler:
    s = sch.get_scheduler()
    s.add(sch.COLLECT_METRICS, collect_metrics, settings.SERVER_METRICS_COLLECT_INTERVAL)
    s.add(sch.DELETE_METRICS, delete_metrics, 300)
    s.add(sch.SUBMITTED_JOBS, process_submitted_jobs, 4, jitter=2, workers=2)
    s.add(sch.RUNNING_JOBS, process_running_jobs, 1, jitter=0.2, workers=2)
    s.add(sch.TERMINATING_JOBS, process_terminating_jobs, 4, jitter=2, workers=2)
    s.add(sch.RUNS, process_runs, 2, jitter=1, workers=2)
    s.add(sch.INSTANCES, process_instances, 4, jitter=2, workers=2)
    s.add(sch.FLEETS, process_fleets, 10, jitter=2)
    s.add(sch.VOLUMES, process_submitted_volumes, 10, jitter=2)
    s.add(sch.GATEWAYS, process_submitted_gateways, 10, jitter=2)
    s.add(sch.GATEWAYS_CONNECTIONS, process_gateways_connections, 15)
    s.add(sch.PLACEMENT_GROUPS, process_placement_groups, 30, jitter=5)
    s.start()
    return s
