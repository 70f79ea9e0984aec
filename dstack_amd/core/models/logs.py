"""Run/job logs and hardware metrics (reference: ``C/models/logs.py``, ``metrics.py``)."""

from __future__ import annotations

from datetime import datetime
from enum import Enum
from typing import List, Optional

from dstack_amd.core.models.common import CoreModel


class LogEventSource(str, Enum):
    STDOUT = "stdout"
    STDERR = "stderr"


class LogEvent(CoreModel):
    timestamp: datetime
    log_source: LogEventSource = LogEventSource.STDOUT
    message: str  # base64-encoded bytes on the wire


class JobSubmissionLogs(CoreModel):
    logs: List[LogEvent]
    next_token: Optional[str] = None


class Metric(CoreModel):
    name: str
    timestamps: List[datetime]
    values: List[float]


class JobMetrics(CoreModel):
    metrics: List[Metric]
