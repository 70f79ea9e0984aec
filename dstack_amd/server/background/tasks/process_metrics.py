"""Hardware-metrics collection every 10 s from each RUNNING job's runner (cgroup CPU/memory +
amdsmi GPU util/VRAM/power/temperature) and TTL cleanup (reference:
``S/background/tasks/process_metrics.py:28-142``)."""

from __future__ import annotations

import concurrent.futures as cf
import logging

from sqlalchemy import select

from dstack_amd.core.models.runs import JobStatus
from dstack_amd.server import settings
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import JobModel
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.server.services import metrics as metrics_services
from dstack_amd.server.services.runner.client import get_runner_client

logger = logging.getLogger(__name__)
MAX_JOBS = 100
BATCH = 10


def collect_metrics() -> bool:
    with session_scope() as s:
        jobs = list(s.execute(select(JobModel).where(JobModel.status == JobStatus.RUNNING.value)
                              .limit(MAX_JOBS)).scalars())
        targets = []
        for j in jobs:
            jpd = jobs_services.job_jpd(j)
            if jpd is None:
                continue
            targets.append((j.id, jpd, jobs_services.job_jrd(j), j.project.ssh_private_key))

    def fetch(t):
        job_id, jpd, jrd, key = t
        try:
            return job_id, get_runner_client(jpd, jrd, key).get_metrics()
        except Exception:  # noqa: BLE001
            return job_id, None

    results = []
    if targets:
        with cf.ThreadPoolExecutor(max_workers=BATCH) as ex:
            results = list(ex.map(fetch, targets))
    with session_scope() as s:
        for job_id, m in results:
            if m:
                job = s.get(JobModel, job_id)
                if job is not None:
                    metrics_services.store_metrics_point(s, job, m)
    return False


def delete_metrics() -> bool:
    with session_scope() as s:
        metrics_services.delete_old_metrics(s, settings.SERVER_METRICS_TTL_SECONDS)
    return False
