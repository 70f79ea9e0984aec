"""Prometheus exposition at ``/metrics`` (the reference lists this as future work —
``docs/blog/posts/monitoring-gpu-usage.md:57-61``; the MI355X build ships it).

Control-plane gauges (runs/jobs/instances by status, per-project) plus the latest amdsmi samples
of every running job (GPU utilisation and VRAM per GPU, CPU and memory), and the scheduler's
per-task run/error counters.  Rendered on request from the DB (no background registry state), so
several server replicas expose consistent numbers.
"""

from __future__ import annotations

import json
from collections import Counter
from typing import List

from sqlalchemy import func, select
from sqlalchemy.orm import Session

from dstack_amd.server.models import InstanceModel, JobMetricsPoint, JobModel, ProjectModel, RunModel


def _esc(v: str) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", " ")


def render(s: Session) -> str:
    out: List[str] = []

    def gauge(name: str, help_: str):
        out.append(f"# HELP {name} {help_}")
        out.append(f"# TYPE {name} gauge")

    projects = {p.id: p.name for p in s.execute(select(ProjectModel)).scalars()}
    gauge("dstack_runs", "Runs by project and status")
    for (pid, st), n in Counter((r.project_id, r.status) for r in s.execute(
            select(RunModel).where(RunModel.deleted == False)).scalars()).items():  # noqa: E712
        out.append(f'dstack_runs{{project="{_esc(projects.get(pid, "?"))}",status="{st}"}} {n}')
    gauge("dstack_jobs", "Job submissions by status")
    for st, n in s.execute(select(JobModel.status, func.count()).group_by(JobModel.status)).all():
        out.append(f'dstack_jobs{{status="{st}"}} {n}')
    gauge("dstack_instances", "Instances by backend and status")
    for (be, st), n in Counter((i.backend or "", i.status) for i in s.execute(
            select(InstanceModel).where(InstanceModel.deleted == False)).scalars()).items():  # noqa: E712
        out.append(f'dstack_instances{{backend="{be}",status="{st}"}} {n}')

    gauge("dstack_job_gpu_util_percent", "Latest GPU utilisation of running jobs (amdsmi)")
    util_lines, mem_lines, cpu_lines, rss_lines = [], [], [], []
    links_lines, xrd_lines, xwr_lines = [], [], []
    for job in s.execute(select(JobModel).where(JobModel.status == "running")).scalars():
        pt = s.execute(select(JobMetricsPoint).where(JobMetricsPoint.job_id == job.id)
                       .order_by(JobMetricsPoint.timestamp_micro.desc())).scalars().first()
        if pt is None:
            continue
        lbl = f'run="{_esc(job.run.run_name)}",job="{_esc(job.job_name)}"'
        for i, u in enumerate(json.loads(pt.gpus_util_percent or "[]")):
            util_lines.append(f'dstack_job_gpu_util_percent{{{lbl},gpu="{i}"}} {u}')
        for i, m in enumerate(json.loads(pt.gpus_memory_usage_bytes or "[]")):
            mem_lines.append(f'dstack_job_gpu_memory_usage_bytes{{{lbl},gpu="{i}"}} {m}')
        for i, e in enumerate(json.loads(pt.gpus_extra or "[]")):
            x = (e or {}).get("xgmi")
            if x:
                links_lines.append(f'dstack_job_gpu_xgmi_links_up{{{lbl},gpu="{i}"}} {x.get("links_up", 0)}')
                xrd_lines.append(f'dstack_job_gpu_xgmi_read_bytes_total{{{lbl},gpu="{i}"}} '
                                 f'{int(x.get("read_kb", 0)) * 1024}')
                xwr_lines.append(f'dstack_job_gpu_xgmi_write_bytes_total{{{lbl},gpu="{i}"}} '
                                 f'{int(x.get("write_kb", 0)) * 1024}')
        cpu_lines.append(f"dstack_job_cpu_usage_micro{{{lbl}}} {pt.cpu_usage_micro or 0}")
        rss_lines.append(f"dstack_job_memory_working_set_bytes{{{lbl}}} {pt.memory_working_set_bytes or 0}")
    out += util_lines
    gauge("dstack_job_gpu_memory_usage_bytes", "Latest VRAM usage of running jobs (amdsmi)")
    out += mem_lines
    out.append("# TYPE dstack_job_cpu_usage_micro counter")
    out += cpu_lines
    gauge("dstack_job_memory_working_set_bytes", "Latest memory working set of running jobs (cgroup)")
    out += rss_lines
    gauge("dstack_job_gpu_xgmi_links_up", "xGMI links up per GPU of running jobs (amdsmi)")
    out += links_lines
    out.append("# TYPE dstack_job_gpu_xgmi_read_bytes_total counter")
    out += xrd_lines
    out.append("# TYPE dstack_job_gpu_xgmi_write_bytes_total counter")
    out += xwr_lines

    from dstack_amd.server.background.scheduler import get_scheduler

    out.append("# TYPE dstack_scheduler_task_runs counter")
    out.append("# TYPE dstack_scheduler_task_errors counter")
    for name, st in get_scheduler().stats().items():
        out.append(f'dstack_scheduler_task_runs{{task="{name}"}} {st["runs"]}')
        out.append(f'dstack_scheduler_task_errors{{task="{name}"}} {st["errors"]}')
    return "\n".join(out) + "\n"
