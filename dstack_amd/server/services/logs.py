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


class LogStorageError(Exception):
    """The log backend cannot be used (bad configuration, missing group, API failure)."""


class CloudWatchLogStorage(LogStorage):
    """CloudWatch Logs over its JSON API (SigV4, no SDK), one stream per
    ``{project}/{run}/{job_submission_id}/{runner|job}``.  Follows the service's PutLogEvents limits
    (reference ``services/logs.py:CloudWatchLogStorage``): a batch holds at most 10,000 events and
    1 MiB (message bytes + 26 per event) and spans at most 24 h; events more than 14 days old or 2 h
    in the future are dropped (both bounds shortened by a 10 min clock-drift margin); a stream that
    vanished (retention) is re-created and the write retried once."""

    EVENT_MAX_COUNT_IN_BATCH = 10000
    BATCH_MAX_SIZE = 1048576
    MESSAGE_MAX_SIZE = 262144
    MESSAGE_OVERHEAD_SIZE = 26
    BATCH_MAX_SPAN = 24 * 3600 * 1000
    CLOCK_DRIFT = 10 * 60 * 1000
    PAST_EVENT_MAX_DELTA = 14 * 24 * 3600 * 1000 - CLOCK_DRIFT
    FUTURE_EVENT_MAX_DELTA = 2 * 3600 * 1000 - CLOCK_DRIFT
    MAX_EMPTY_BACKWARD_PAGES = 10

    def __init__(self, group: str, region: Optional[str] = None, client=None, credentials=None):
        import httpx

        self.group = group
        self.region = region or os.getenv("DSTACK_SERVER_CLOUDWATCH_LOG_REGION") or os.getenv("AWS_REGION", "us-east-1")
        self.url = f"https://logs.{self.region}.amazonaws.com/"
        creds = credentials or (os.getenv("AWS_ACCESS_KEY_ID"), os.getenv("AWS_SECRET_ACCESS_KEY"),
                                os.getenv("AWS_SESSION_TOKEN"))
        if not creds[0] or not creds[1]:
            raise LogStorageError("CloudWatch Logs: no AWS credentials (AWS_ACCESS_KEY_ID / AWS_SECRET_ACCESS_KEY)")
        self._creds = creds
        self.http = client or httpx.Client(timeout=30)
        self._streams: set = set()
        try:
            self._call("DescribeLogStreams", {"logGroupName": group, "limit": 1})
        except _CloudWatchError as e:
            if e.not_found:
                raise LogStorageError(f"LogGroup '{group}' does not exist") from e
            raise LogStorageError(f"CloudWatch Logs error: {e}") from e

    # ---- transport ------------------------------------------------------------------------------
    def _call(self, target: str, body: dict) -> dict:
        import httpx

        from dstack_amd.core.backends.clouds.common import sigv4_headers

        data = json.dumps(body).encode()
        h = sigv4_headers("POST", self.url, self.region, "logs", self._creds[0], self._creds[1], data,
                          self._creds[2], extra_headers={"x-amz-target": f"Logs_20140328.{target}",
                                                         "content-type": "application/x-amz-json-1.1"})
        try:
            r = self.http.post(self.url, content=data, headers=h)
        except httpx.HTTPError as e:
            raise _CloudWatchError(target, "RequestError", str(e)) from e
        if r.status_code >= 400:
            try:
                err = r.json()
            except ValueError:
                err = {}
            code = str(err.get("__type", "")).rsplit("#", 1)[-1] or f"HTTP{r.status_code}"
            raise _CloudWatchError(target, code, err.get("message") or r.text[:300])
        return r.json() if r.content else {}

    @staticmethod
    def _stream(project, run_name, sub_id, kind):
        return f"{project}/{run_name}/{sub_id}/{kind}"

    # ---- streams --------------------------------------------------------------------------------
    def _ensure_stream(self, name: str, force: bool = False) -> None:
        if not force and name in self._streams:
            return
        d = self._call("DescribeLogStreams", {"logGroupName": self.group, "logStreamNamePrefix": name})
        if not any(st.get("logStreamName") == name for st in d.get("logStreams", [])):
            try:
                self._call("CreateLogStream", {"logGroupName": self.group, "logStreamName": name})
            except _CloudWatchError as e:
                if e.code != "ResourceAlreadyExistsException":
                    raise
        self._streams.add(name)

    # ---- write ----------------------------------------------------------------------------------
    def write_logs(self, project, run_name, job_submission_id, runner_logs, job_logs):
        for kind, events in (("runner", runner_logs), ("job", job_logs)):
            if events:
                self._write(self._stream(project, run_name, job_submission_id, kind), events)

    def _write(self, stream: str, events: List[dict]) -> None:
        try:
            self._ensure_stream(stream)
            try:
                self._put(stream, events)
                return
            except _CloudWatchError as e:
                if not e.not_found:
                    raise
            self._ensure_stream(stream, force=True)  # deleted by retention: our cache was stale
            self._put(stream, events)
        except _CloudWatchError as e:
            raise LogStorageError(f"CloudWatch Logs error: {e}") from e

    def _put(self, stream: str, events: List[dict]) -> None:
        ordered = sorted(events, key=lambda e: int(e["timestamp"]))  # stable: runner order within a ms
        for batch in self.batches(ordered):
            self._call("PutLogEvents", {"logGroupName": self.group, "logStreamName": stream, "logEvents": batch})

    def batches(self, events: List[dict], now_ms: Optional[int] = None):
        """Chronological events -> PutLogEvents batches within the service limits."""
        import time

        now = int(time.time() * 1000) if now_ms is None else now_ms
        batch: List[dict] = []
        size = 0
        first = None
        for e in events:
            msg = e.get("message") or ""
            if not msg:
                continue
            ts = int(e["timestamp"])
            if now - ts > self.PAST_EVENT_MAX_DELTA or ts - now > self.FUTURE_EVENT_MAX_DELTA:
                continue  # CloudWatch rejects the whole request for one such event
            msize = len(msg.encode()) + self.MESSAGE_OVERHEAD_SIZE
            if msize > self.MESSAGE_MAX_SIZE:
                continue
            if batch and (ts - first > self.BATCH_MAX_SPAN or size + msize > self.BATCH_MAX_SIZE or
                          len(batch) >= self.EVENT_MAX_COUNT_IN_BATCH):
                yield batch
                batch, size, first = [], 0, None
            if first is None:
                first = ts
            batch.append({"timestamp": ts, "message": msg})
            size += msize
        if batch:
            yield batch

    # ---- read -----------------------------------------------------------------------------------
    def poll_logs(self, project, run_name, job_submission_id, start_time=None, end_time=None, descending=False,
                  limit=1000, diagnose=False) -> JobSubmissionLogs:
        stream = self._stream(project, run_name, job_submission_id, "runner" if diagnose else "job")
        body = {"logGroupName": self.group, "logStreamName": stream, "limit": limit, "startFromHead": not descending}
        if start_time is not None:
            # start is inclusive in CloudWatch; callers page with the last timestamp they saw
            body["startTime"] = int(_aware(start_time).timestamp() * 1000) + 1
        if end_time is not None:
            body["endTime"] = int(_aware(end_time).timestamp() * 1000)
        try:
            raw = self._get_events(body)
        except _CloudWatchError as e:
            if e.not_found:
                return JobSubmissionLogs(logs=[])
            raise LogStorageError(f"CloudWatch Logs error: {e}") from e
        if descending:
            raw = list(reversed(raw))  # CloudWatch returns chronological order either way
        events = [LogEvent(timestamp=datetime.fromtimestamp(e["timestamp"] / 1000, tz=timezone.utc),
                           message=e["message"]) for e in raw]
        next_token = events[-1].timestamp.isoformat() if events and len(events) == limit else None
        return JobSubmissionLogs(logs=events, next_token=next_token)

    def _get_events(self, body: dict) -> List[dict]:
        d = self._call("GetLogEvents", body)
        events = d.get("events", [])
        if body["startFromHead"] or events:
            return events
        # reading backwards, GetLogEvents may return empty pages before the newest events: follow
        # nextBackwardToken until events appear or the token stops moving (bounded)
        token = d.get("nextBackwardToken")
        for _ in range(self.MAX_EMPTY_BACKWARD_PAGES):
            d = self._call("GetLogEvents", dict(body, nextToken=token))
            events = d.get("events", [])
            if events or d.get("nextBackwardToken") == token:
                return events
            token = d.get("nextBackwardToken")
        return []


class _CloudWatchError(Exception):
    def __init__(self, target: str, code: str, message: str):
        super().__init__(f"{target}: {code}: {message}")
        self.code = code

    @property
    def not_found(self) -> bool:
        return self.code == "ResourceNotFoundException"


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
