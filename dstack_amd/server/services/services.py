"""Service runs: registration (gateway or in-server proxy) and autoscaling (reference:
``S/services/services/__init__.py:39-231``, ``autoscalers.py:38-126``).

Autoscalers:
* ``ManualScaler`` — clip the desired count to ``replicas`` min..max;
* ``RPSAutoscaler`` — target tracking on requests/s per replica (60 s window) with scale-up/down
  delays, fed by gateway stats or the in-server proxy's request counters;
* ``GPUUtilAutoscaler`` (MI355X addition) — target tracking on the mean amdsmi GPU busy % of the
  replicas (from ``job_metrics_points``), for LLM serving whose saturation shows in the GPU.
"""

from __future__ import annotations

import json
import math
import threading
import time
from abc import ABC, abstractmethod
from collections import defaultdict, deque
from dataclasses import dataclass
from datetime import datetime, timedelta
from typing import Deque, Dict, List, Optional, Tuple

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import GatewayError, ResourceNotExistsError
from dstack_amd.core.models.configurations import ServiceConfiguration
from dstack_amd.core.models.runs import RunSpec, ServiceModelSpec, ServiceSpec
from dstack_amd.core.models.services import ScalingSpec
from dstack_amd.server.models import GatewayModel, JobMetricsPoint, JobModel, RunModel
from dstack_amd.utils.common import get_current_datetime


# ---------------------------------------------------------------------------------------------
# registration
# ---------------------------------------------------------------------------------------------
def register_service(s: Session, run: RunModel):
    spec = RunSpec.model_validate_json(run.run_spec)
    conf: ServiceConfiguration = spec.configuration  # type: ignore[assignment]
    project = run.project
    gateway = None
    if conf.gateway is not False:
        q = select(GatewayModel).where(GatewayModel.project_id == project.id)
        if isinstance(conf.gateway, str):
            gateway = s.execute(q.where(GatewayModel.name == conf.gateway)).scalar_one_or_none()
            if gateway is None:
                raise GatewayError(f"Gateway {conf.gateway} does not exist")
        elif project.default_gateway_id:
            gateway = s.get(GatewayModel, project.default_gateway_id)
    if gateway is not None and gateway.wildcard_domain:
        host = f"{run.run_name}.{gateway.wildcard_domain}"
        scheme = "https" if conf.https else "http"
        url = f"{scheme}://{host}"
        model = None
        if conf.model is not None:
            model = ServiceModelSpec(name=conf.model.name, base_url=f"{scheme}://gateway.{gateway.wildcard_domain}",
                                     type=conf.model.type)
        run.gateway_id = gateway.id
        svc = ServiceSpec(url=url, model=model, options={"gateway": gateway.name})
        from dstack_amd.server.services.gateways import gateway_register_service

        gateway_register_service(s, run)
    else:
        from dstack_amd.server import settings

        if settings.FORBID_SERVICES_WITHOUT_GATEWAY:
            raise ResourceNotExistsError("This dstack server forbids services without a gateway. "
                                         "Please configure a gateway.")
        # (the in-server proxy counts requests too, so rps autoscaling works without a gateway)
        url = f"/proxy/services/{project.name}/{run.run_name}/"
        model = None
        if conf.model is not None:
            model = ServiceModelSpec(name=conf.model.name, base_url=f"/proxy/models/{project.name}/",
                                     type=conf.model.type)
        svc = ServiceSpec(url=url, model=model)
    run.service_spec = svc.model_dump_json()


def unregister_service(s: Session, run: RunModel):
    get_request_stats().forget(run.id)
    if run.gateway_id is not None:
        from dstack_amd.server.services.gateways import gateway_unregister_service

        gateway_unregister_service(s, run)


# ---------------------------------------------------------------------------------------------
# request statistics (in-server proxy and gateway stats land here)
# ---------------------------------------------------------------------------------------------
class RequestStats:
    """Per-service request timestamps kept for the largest window (300 s)."""

    WINDOW = 300.0

    def __init__(self):
        self._lock = threading.Lock()
        self._events: Dict[object, Deque[Tuple[float, float]]] = defaultdict(deque)
        self._external: Dict[object, Tuple[float, float, float]] = {}

    def record(self, service_id, duration_s: float = 0.0, ts: Optional[float] = None):
        ts = ts or time.time()
        with self._lock:
            q = self._events[service_id]
            q.append((ts, duration_s))
            while q and q[0][0] < ts - self.WINDOW:
                q.popleft()

    def set_external(self, service_id, rps: float, mean_request_time: float):
        """Aggregates reported by a gateway (its nginx/data plane saw the requests, not us)."""
        with self._lock:
            self._external[service_id] = (time.time(), rps, mean_request_time)

    def _external_fresh(self, service_id):
        e = self._external.get(service_id)
        return e if e is not None and time.time() - e[0] < 120 else None

    def rps(self, service_id, window: float = 60.0) -> float:
        now = time.time()
        with self._lock:
            q = self._events.get(service_id)
            n = sum(1 for t, _ in q if t >= now - window) if q else 0
            ext = self._external_fresh(service_id)
        return n / window + (ext[1] if ext else 0.0)

    def mean_request_time(self, service_id, window: float = 60.0) -> float:
        now = time.time()
        with self._lock:
            d = [x for t, x in self._events.get(service_id, ()) if t >= now - window]
        return sum(d) / len(d) if d else 0.0

    def forget(self, service_id):
        with self._lock:
            self._events.pop(service_id, None)
            self._external.pop(service_id, None)


_stats = RequestStats()


def get_request_stats() -> RequestStats:
    return _stats


# ---------------------------------------------------------------------------------------------
# autoscalers
# ---------------------------------------------------------------------------------------------
@dataclass
class ReplicaInfo:
    active: bool
    timestamp: datetime  # when the replica last changed state


class BaseServiceScaler(ABC):
    @abstractmethod
    def scale(self, replicas: List[ReplicaInfo], metric_value: Optional[float]) -> int:
        """Return the replica delta."""


class ManualScaler(BaseServiceScaler):
    def __init__(self, min_replicas: int, max_replicas: int):
        self.min, self.max = min_replicas, max_replicas

    def scale(self, replicas: List[ReplicaInfo], metric_value: Optional[float]) -> int:
        active = sum(1 for r in replicas if r.active)
        return min(self.max, max(self.min, active)) - active


class _TargetTracking(BaseServiceScaler):
    def __init__(self, min_replicas: int, max_replicas: int, target: float, scale_up_delay: int,
                 scale_down_delay: int):
        self.min, self.max, self.target = min_replicas, max_replicas, target
        self.up_delay, self.down_delay = scale_up_delay, scale_down_delay

    def desired(self, active: int, metric_value: float) -> int:
        raise NotImplementedError

    def scale(self, replicas: List[ReplicaInfo], metric_value: Optional[float]) -> int:
        active = [r for r in replicas if r.active]
        n = len(active)
        if metric_value is None:
            return ManualScaler(self.min, self.max).scale(replicas, None)
        want = min(self.max, max(self.min, self.desired(n, metric_value)))
        if want == n:
            return 0
        last = max((r.timestamp for r in replicas), default=None)
        now = get_current_datetime()
        if want > n:
            if n == 0 or last is None or now - last >= timedelta(seconds=self.up_delay):
                return want - n
            return 0
        if last is None or now - last >= timedelta(seconds=self.down_delay):
            return want - n
        return 0


class RPSAutoscaler(_TargetTracking):
    """replicas = ceil(total_rps / target)."""

    def desired(self, active: int, rps: float) -> int:
        return math.ceil(rps / self.target) if rps > 0 else self.min


class GPUUtilAutoscaler(_TargetTracking):
    """replicas = ceil(active * mean_util / target) (target in %, e.g. 75)."""

    def desired(self, active: int, util: float) -> int:
        if active == 0:
            return self.min or 1
        return max(1, math.ceil(active * util / self.target))


def get_service_scaler(conf: ServiceConfiguration) -> BaseServiceScaler:
    lo, hi = conf.replicas.min or 0, conf.replicas.max
    sc: Optional[ScalingSpec] = conf.scaling
    if sc is None:
        return ManualScaler(lo, hi)
    cls = RPSAutoscaler if sc.metric == "rps" else GPUUtilAutoscaler
    return cls(lo, hi, sc.target, int(sc.scale_up_delay), int(sc.scale_down_delay))


def service_metric_value(s: Session, run: RunModel, conf: ServiceConfiguration) -> Optional[float]:
    if conf.scaling is None:
        return None
    if conf.scaling.metric == "rps":
        return get_request_stats().rps(run.id)
    # gpu_util: the measured load -- each running job's latest amdsmi util sample of the last
    # 2 minutes (mean over its GPUs), summed and spread over every running job.  A job without a
    # recent sample (a replica that just started) counts as idle, so the scaler sizes for the load
    # it can see: replicas = ceil(sum(util) / target).  No sample at all: no signal, no scaling.
    since = int((time.time() - 120) * 1e6)
    utils: List[float] = []
    running = 0
    for j in run.jobs:
        if j.status != "running":
            continue
        running += 1
        pt = s.execute(select(JobMetricsPoint).where(JobMetricsPoint.job_id == j.id,
                                                     JobMetricsPoint.timestamp_micro >= since)
                       .order_by(JobMetricsPoint.timestamp_micro.desc())).scalars().first()
        if pt is not None:
            vals = json.loads(pt.gpus_util_percent or "[]")
            if vals:
                utils.append(sum(vals) / len(vals))
    return sum(utils) / running if utils else None


def register_replica(s: Session, run: RunModel, job: JobModel):
    """The in-server proxy resolves replicas from the DB on each request; gateways get pushed
    the new upstream (``register_replica``)."""
    if run.gateway_id is not None:
        from dstack_amd.server.services.gateways import gateway_register_replica

        gateway_register_replica(s, run, job)


def unregister_replica(s: Session, run: RunModel, job: JobModel):
    if run.gateway_id is not None:
        from dstack_amd.server.services.gateways import gateway_unregister_replica

        gateway_unregister_replica(s, run, job)
