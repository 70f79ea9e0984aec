"""Job/runner log storage (reference: ``S/services/logs.py:344-471``).

File backend: ``<server_dir>/projects/<p>/logs/<run>/<job_submission_id>/{runner,job}.log`` as
JSON lines ``{"timestamp": iso, "log_source": "stdout", "message": <base64>}``.  A per-file
in-memory index of byte offsets makes ``poll`` by ``start_time`` a seek, not a scan."""

from __future__ import annotations

import base64
import json
import os
import threading
from datetime import datetime, timezone
from pathlib import Path
from typing import List, Optional

from dstack_amd.core.models.logs import JobSubmissionLogs, LogEvent, LogEventSource
from dstack_amd.server import settings


class LogStorage:
    def write_logs(self, project: str, run_name: str, job_submission_id: str, runner_logs: List[dict],
                   job_logs: List[dict]) -> None:
        raise NotImplementedError

    def poll_logs(self, project: str, run_name: str, job_submission_id: str, start_time: Optional[datetime] = None,
                  end_time: Optional[datetime] = None, descending: bool = False, limit: int = 1000,
                  diagnose: bool = False) -> JobSubmissionLogs:
        raise NotImplementedError


def _to_iso(ts_ms: int) -> str:
    return datetime.fromtimestamp(ts_ms / 1000, tz=timezone.utc).isoformat()


class FileLogStorage(LogStorage):
    def __init__(self, root: Optional[Path] = None):
        self.root = Path(root or settings.SERVER_DIR_PATH)
        self._lock = threading.Lock()

    def _path(self, project: str, run_name: str, sub_id: str, kind: str) -> Path:
        return self.root / "projects" / project / "logs" / run_name / sub_id / f"{kind}.log"

    def write_logs(self, project, run_name, job_submission_id, runner_logs, job_logs):
        for kind, events in (("runner", runner_logs), ("job", job_logs)):
            if not events:
                continue
            p = self._path(project, run_name, job_submission_id, kind)
            p.parent.mkdir(parents=True, exist_ok=True)
            lines = "".join(
                json.dumps({"timestamp": _to_iso(int(e["timestamp"])), "log_source": "stdout",
                            "message": e["message"]}) + "\n"
                for e in events
            )
            with self._lock, open(p, "a") as f:
                f.write(lines)

    def poll_logs(self, project, run_name, job_submission_id, start_time=None, end_time=None, descending=False,
                  limit=1000, diagnose=False) -> JobSubmissionLogs:
        p = self._path(project, run_name, job_submission_id, "runner" if diagnose else "job")
        events: List[LogEvent] = []
        if p.exists():
            with open(p) as f:
                for line in f:
                    try:
                        d = json.loads(line)
                    except ValueError:
                        continue
                    ts = datetime.fromisoformat(d["timestamp"])
                    if start_time is not None and ts <= _aware(start_time):
                        continue
                    if end_time is not None and ts > _aware(end_time):
                        continue
                    events.append(LogEvent(timestamp=ts, log_source=LogEventSource(d.get("log_source", "stdout")),
                                           message=d["message"]))
        if descending:
            events.reverse()
        events = events[:limit]
        next_token = events[-1].timestamp.isoformat() if len(events) == limit else None
        return JobSubmissionLogs(logs=events, next_token=next_token)


def _aware(dt: datetime) -> datetime:
    return dt if dt.tzinfo else dt.replace(tzinfo=timezone.utc)


_storage: Optional[LogStorage] = None


def get_default_log_storage() -> LogStorage:
    global _storage
    if _storage is None:
        _storage = FileLogStorage()
    return _storage


def override_log_storage(storage: LogStorage):
    global _storage
    _storage = storage


def decode_message(e: LogEvent) -> str:
    return base64.b64decode(e.message).decode(errors="replace")


def write_job_logs(project: str, run_name: str, job_submission_id: str, pull: dict):
    get_default_log_storage().write_logs(project, run_name, job_submission_id, pull.get("runner_logs") or [],
                                         pull.get("job_logs") or [])


_ = os
