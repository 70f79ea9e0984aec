"""Job/runner log storage (reference: ``S/services/logs.py:65-471``).

* File backend: ``<server_dir>/projects/<p>/logs/<run>/<job_submission_id>/{runner,job}.log`` as
  JSON lines ``{"timestamp": iso, "log_source": "stdout", "message": <base64>}``.  An incremental
  per-file index (timestamp -> byte offset, extended as the file grows) turns ``poll`` by
  ``start_time`` into a bisect + seek, so following a long training log stays O(new lines).
* CloudWatch backend (``DSTACK_SERVER_CLOUDWATCH_LOG_GROUP``): PutLogEvents / GetLogEvents over
  the JSON API with SigV4 (no boto3); one stream per ``{project}/{run}/{job_submission_id}/{kind}``."""

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
        self._idx: dict = {}

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

    def _index(self, p: Path):
        """(timestamps, offsets) of every line, extended from the last indexed size."""
        st = self._idx.get(p)
        if st is None:
            st = self._idx[p] = ([], [], 0)
        ts_list, offs, end = st
        size = p.stat().st_size
        if size < end:  # truncated/rotated: rebuild
            ts_list, offs, end = [], [], 0
        if size > end:
            with open(p, "rb") as f:
                f.seek(end)
                pos = end
                for raw in f:
                    if not raw.endswith(b"\n"):
                        break
                    try:
                        ts_list.append(datetime.fromisoformat(json.loads(raw)["timestamp"]).timestamp())
                        offs.append(pos)
                    except (ValueError, KeyError):
                        pass
                    pos += len(raw)
                end = pos
        self._idx[p] = (ts_list, offs, end)
        return ts_list, offs, end

    def poll_logs(self, project, run_name, job_submission_id, start_time=None, end_time=None, descending=False,
                  limit=1000, diagnose=False) -> JobSubmissionLogs:
        import bisect

        p = self._path(project, run_name, job_submission_id, "runner" if diagnose else "job")
        events: List[LogEvent] = []
        if p.exists():
            with self._lock:
                ts_list, offs, end = self._index(p)
            lo = bisect.bisect_right(ts_list, _aware(start_time).timestamp()) if start_time is not None else 0
            # (start_time, end_time) is exclusive at both ends: callers page with the last timestamp
            hi = bisect.bisect_left(ts_list, _aware(end_time).timestamp()) if end_time is not None else len(ts_list)
            if descending:
                lo = max(lo, hi - limit)
            else:
                hi = min(hi, lo + limit)
            if lo < hi:
                with open(p, "rb") as f:
                    f.seek(offs[lo])
                    for _ in range(hi - lo):
                        d = json.loads(f.readline())
                        events.append(LogEvent(timestamp=datetime.fromisoformat(d["timestamp"]),
                                               log_source=LogEventSource(d.get("log_source", "stdout")),
                                               message=d["message"]))
        if descending:
            events.reverse()
        next_token = events[-1].timestamp.isoformat() if len(events) == limit else None
        return JobSubmissionLogs(logs=events, next_token=next_token)


class CloudWatchLogStorage(LogStorage):
    def __init__(self, group: str, region: Optional[str] = None, client=None):
        import httpx

        self.group = group
        self.region = region or os.getenv("DSTACK_SERVER_CLOUDWATCH_LOG_REGION") or os.getenv("AWS_REGION", "us-east-1")
        self.url = f"https://logs.{self.region}.amazonaws.com/"
        self.http = client or httpx.Client(timeout=30)
        self._streams = set()

    def _call(self, target: str, body: dict) -> dict:
        from dstack_amd.core.backends.clouds.common import sigv4_headers

        data = json.dumps(body).encode()
        h = sigv4_headers("POST", self.url, self.region, "logs", os.getenv("AWS_ACCESS_KEY_ID", ""),
                          os.getenv("AWS_SECRET_ACCESS_KEY", ""), data, os.getenv("AWS_SESSION_TOKEN"),
                          extra_headers={"x-amz-target": f"Logs_20140328.{target}",
                                         "content-type": "application/x-amz-json-1.1"})
        r = self.http.post(self.url, content=data, headers=h)
        if r.status_code >= 400 and "ResourceAlreadyExistsException" not in r.text:
            raise RuntimeError(f"CloudWatch {target}: {r.status_code} {r.text[:300]}")
        return r.json() if r.content else {}

    @staticmethod
    def _stream(project, run_name, sub_id, kind):
        return f"{project}/{run_name}/{sub_id}/{kind}"

    def write_logs(self, project, run_name, job_submission_id, runner_logs, job_logs):
        for kind, events in (("runner", runner_logs), ("job", job_logs)):
            if not events:
                continue
            stream = self._stream(project, run_name, job_submission_id, kind)
            if stream not in self._streams:
                self._call("CreateLogStream", {"logGroupName": self.group, "logStreamName": stream})
                self._streams.add(stream)
            # PutLogEvents: chronological, <= 10k events per batch
            evs = sorted(events, key=lambda e: int(e["timestamp"]))
            for i in range(0, len(evs), 10000):
                self._call("PutLogEvents", {"logGroupName": self.group, "logStreamName": stream, "logEvents": [
                    {"timestamp": int(e["timestamp"]), "message": e["message"]} for e in evs[i:i + 10000]]})

    def poll_logs(self, project, run_name, job_submission_id, start_time=None, end_time=None, descending=False,
                  limit=1000, diagnose=False) -> JobSubmissionLogs:
        body = {"logGroupName": self.group, "limit": limit, "startFromHead": not descending,
                "logStreamName": self._stream(project, run_name, job_submission_id, "runner" if diagnose else "job")}
        if start_time is not None:
            body["startTime"] = int(_aware(start_time).timestamp() * 1000) + 1
        if end_time is not None:
            body["endTime"] = int(_aware(end_time).timestamp() * 1000)
        try:
            d = self._call("GetLogEvents", body)
        except RuntimeError as e:
            if "ResourceNotFoundException" in str(e):
                return JobSubmissionLogs(logs=[])
            raise
        events = [LogEvent(timestamp=datetime.fromtimestamp(e["timestamp"] / 1000, tz=timezone.utc),
                           message=e["message"]) for e in d.get("events", [])]
        next_token = events[-1].timestamp.isoformat() if len(events) == limit else None
        return JobSubmissionLogs(logs=events, next_token=next_token)


def _aware(dt: datetime) -> datetime:
    return dt if dt.tzinfo else dt.replace(tzinfo=timezone.utc)


_storage: Optional[LogStorage] = None


def get_default_log_storage() -> LogStorage:
    global _storage
    if _storage is None:
        group = os.getenv("DSTACK_SERVER_CLOUDWATCH_LOG_GROUP") or settings.SERVER_CLOUDWATCH_LOG_GROUP
        _storage = CloudWatchLogStorage(group) if group else FileLogStorage()
    return _storage


def override_log_storage(storage: LogStorage):
    global _storage
    _storage = storage


def decode_message(e: LogEvent) -> str:
    return base64.b64decode(e.message).decode(errors="replace")


def write_job_logs(project: str, run_name: str, job_submission_id: str, pull: dict):
    get_default_log_storage().write_logs(project, run_name, job_submission_id, pull.get("runner_logs") or [],
                                         pull.get("job_logs") or [])
