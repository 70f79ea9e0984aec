"""Job hardware metrics (reference: ``S/services/metrics.py:13-113``): computed from the last two
``job_metrics_points``; AMD additions from amdsmi: GPU power (W), temperature (°C), HBM controller
activity (%) and xGMI -- links up, and read / write throughput (bytes/s) derived from the
accumulated per-link traffic counters of consecutive samples."""

from __future__ import annotations

import json
from datetime import datetime, timezone
from typing import List, Optional

from sqlalchemy import delete, select
from sqlalchemy.orm import Session

from dstack_amd.core.models.logs import JobMetrics, Metric
from dstack_amd.server.models import JobMetricsPoint, JobModel


def _ts(micro: int) -> datetime:
    return datetime.fromtimestamp(micro / 1e6, tz=timezone.utc)


def get_job_metrics(s: Session, job: JobModel, limit: int = 2) -> JobMetrics:
    pts = list(s.execute(select(JobMetricsPoint).where(JobMetricsPoint.job_id == job.id)
                         .order_by(JobMetricsPoint.timestamp_micro.desc()).limit(max(2, limit))).scalars())
    pts.reverse()
    if len(pts) < 2:
        return JobMetrics(metrics=[])
    return JobMetrics(metrics=_calculate(pts))


def _calculate(pts: List[JobMetricsPoint]) -> List[Metric]:
    ts, cpu, mem, ws = [], [], [], []
    gpus_mem: List[List[float]] = []
    gpus_util: List[List[float]] = []
    gpus_power: List[List[float]] = []
    gpus_temp: List[List[float]] = []
    gpus_hbm: List[List[float]] = []
    xgmi_rd: List[List[float]] = []
    xgmi_wr: List[List[float]] = []
    xgmi_up: List[List[float]] = []
    for prev, cur in zip(pts, pts[1:]):
        ts.append(_ts(cur.timestamp_micro))
        dt = max(1, cur.timestamp_micro - prev.timestamp_micro)
        cpu.append(max(0.0, (cur.cpu_usage_micro - prev.cpu_usage_micro) / dt * 100))
        mem.append(float(cur.memory_usage_bytes))
        ws.append(float(cur.memory_working_set_bytes))
        gm = json.loads(cur.gpus_memory_usage_bytes or "[]")
        gu = json.loads(cur.gpus_util_percent or "[]")
        gp = json.loads(cur.gpus_power_watts or "[]")
        gt = json.loads(cur.gpus_temperature_c or "[]")
        for arr, vals in ((gpus_mem, gm), (gpus_util, gu), (gpus_power, gp), (gpus_temp, gt)):
            while len(arr) < len(vals):
                arr.append([])
            for i, v in enumerate(vals):
                arr[i].append(float(v))
        ex_prev = json.loads(prev.gpus_extra or "[]")
        ex_cur = json.loads(cur.gpus_extra or "[]")
        for i, e in enumerate(ex_cur):
            for arr in (gpus_hbm, xgmi_rd, xgmi_wr, xgmi_up):
                while len(arr) <= i:
                    arr.append([])
            if e.get("mem_activity_percent") is not None:
                gpus_hbm[i].append(float(e["mem_activity_percent"]))
            x = e.get("xgmi")
            if not x:
                continue
            xgmi_up[i].append(float(x.get("links_up", 0)))
            px = (ex_prev[i].get("xgmi") if i < len(ex_prev) else None) or {}
            if px:  # counters are cumulative KiB: rate between the two samples (reset -> 0)
                secs = dt / 1e6
                xgmi_rd[i].append(max(0.0, (x.get("read_kb", 0) - px.get("read_kb", 0)) * 1024 / secs))
                xgmi_wr[i].append(max(0.0, (x.get("write_kb", 0) - px.get("write_kb", 0)) * 1024 / secs))
    metrics = [
        Metric(name="cpu_usage_percent", timestamps=ts, values=cpu),
        Metric(name="memory_usage_bytes", timestamps=ts, values=mem),
        Metric(name="memory_working_set_bytes", timestamps=ts, values=ws),
        Metric(name="gpus_detected_num", timestamps=ts, values=[float(len(gpus_util))] * len(ts)),
    ]
    for i, v in enumerate(gpus_mem):
        metrics.append(Metric(name=f"gpu_memory_usage_bytes_gpu{i}", timestamps=ts[-len(v):], values=v))
    for i, v in enumerate(gpus_util):
        metrics.append(Metric(name=f"gpu_util_percent_gpu{i}", timestamps=ts[-len(v):], values=v))
    for i, v in enumerate(gpus_power):
        metrics.append(Metric(name=f"gpu_power_watts_gpu{i}", timestamps=ts[-len(v):], values=v))
    for i, v in enumerate(gpus_temp):
        metrics.append(Metric(name=f"gpu_temperature_c_gpu{i}", timestamps=ts[-len(v):], values=v))
    for prefix, series in (("gpu_hbm_activity_percent", gpus_hbm), ("gpu_xgmi_links_up", xgmi_up),
                           ("gpu_xgmi_read_bytes_per_s", xgmi_rd), ("gpu_xgmi_write_bytes_per_s", xgmi_wr)):
        for i, v in enumerate(series):
            if v:
                metrics.append(Metric(name=f"{prefix}_gpu{i}", timestamps=ts[-len(v):], values=v))
    return metrics


def store_metrics_point(s: Session, job: JobModel, m: dict):
    import uuid

    gpus = m.get("gpus") or []
    s.add(JobMetricsPoint(
        id=uuid.uuid4(), job_id=job.id, timestamp_micro=int(m.get("timestamp_micro") or 0),
        cpu_usage_micro=int(m.get("cpu_usage_micro") or 0), memory_usage_bytes=int(m.get("memory_usage_bytes") or 0),
        memory_working_set_bytes=int(m.get("memory_working_set_bytes") or 0),
        gpus_memory_usage_bytes=json.dumps([g.get("gpu_memory_usage_bytes", 0) for g in gpus]),
        gpus_util_percent=json.dumps([g.get("gpu_util_percent", 0) for g in gpus]),
        gpus_power_watts=json.dumps([g.get("gpu_power_watts", 0) for g in gpus]),
        gpus_temperature_c=json.dumps([g.get("gpu_temperature_c", 0) for g in gpus]),
        gpus_extra=json.dumps([{"mem_activity_percent": g.get("gpu_mem_activity_percent"), "xgmi": g.get("xgmi")}
                               for g in gpus]),
    ))


def delete_old_metrics(s: Session, ttl_seconds: int, now_micro: Optional[int] = None):
    import time

    now_micro = now_micro or int(time.time() * 1e6)
    s.execute(delete(JobMetricsPoint).where(JobMetricsPoint.timestamp_micro < now_micro - ttl_seconds * 1_000_000))
