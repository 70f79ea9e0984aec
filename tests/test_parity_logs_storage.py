"""Log storage backends, case by case against the reference's ``services/test_logs.py`` (mapping:
``docs/reference/test-parity.md``): the file backend's round trip and the CloudWatch backend against a
stand-in of the CloudWatch Logs JSON API (group check at start, stream create/cache/recreate,
forward / backward polling with the empty-page workaround, request parameters, error mapping,
PutLogEvents batching by count, size and time span, past/future event filtering)."""

from __future__ import annotations

import base64
import json
import time
from datetime import datetime, timedelta, timezone
from typing import Dict, List

import httpx
import pytest

from dstack_amd.server.services.logs import CloudWatchLogStorage, FileLogStorage, LogStorageError

CREDS = ("AKIATEST", "secret", None)


class FakeCloudWatch:
    """In-memory CloudWatch Logs: {group: {stream: [events]}}; records every request."""

    def __init__(self, groups=("dstack",)):
        self.groups: Dict[str, Dict[str, List[dict]]] = {g: {} for g in groups}
        self.requests: List[tuple] = []
        self.fail: Dict[str, tuple] = {}  # target -> (status, __type)
        self.backward_empty_pages = 0

    def client(self):
        return httpx.Client(transport=httpx.MockTransport(self.handle))

    def _err(self, status, kind, msg="error"):
        return httpx.Response(status, json={"__type": f"com.amazonaws.logs#{kind}", "message": msg})

    def handle(self, req: httpx.Request) -> httpx.Response:
        target = req.headers["x-amz-target"].split(".", 1)[1]
        body = json.loads(req.content)
        self.requests.append((target, body))
        assert req.headers["authorization"].startswith("AWS4-HMAC-SHA256")
        if target in self.fail:
            status, kind = self.fail[target]
            return self._err(status, kind)
        group = self.groups.get(body.get("logGroupName"))
        if group is None:
            return self._err(400, "ResourceNotFoundException", "The specified log group does not exist.")
        if target == "DescribeLogStreams":
            prefix = body.get("logStreamNamePrefix", "")
            names = [n for n in group if n.startswith(prefix)][: body.get("limit", 50)]
            return httpx.Response(200, json={"logStreams": [{"logStreamName": n} for n in names]})
        if target == "CreateLogStream":
            if body["logStreamName"] in group:
                return self._err(400, "ResourceAlreadyExistsException")
            group[body["logStreamName"]] = []
            return httpx.Response(200, json={})
        stream = group.get(body.get("logStreamName"))
        if stream is None:
            return self._err(400, "ResourceNotFoundException", "The specified log stream does not exist.")
        if target == "PutLogEvents":
            ts = [e["timestamp"] for e in body["logEvents"]]
            assert ts == sorted(ts), "PutLogEvents needs chronological events"
            assert len(ts) <= 10000 and ts[-1] - ts[0] <= 24 * 3600 * 1000
            assert sum(len(e["message"]) + 26 for e in body["logEvents"]) <= 1048576
            stream.extend(body["logEvents"])
            return httpx.Response(200, json={"nextSequenceToken": "x"})
        if target == "GetLogEvents":
            evs = [e for e in stream if e["timestamp"] >= body.get("startTime", 0)
                   and e["timestamp"] < body.get("endTime", 1 << 62)]
            if not body["startFromHead"] and "nextToken" not in body and self.backward_empty_pages:
                return httpx.Response(200, json={"events": [], "nextBackwardToken": "b/1", "nextForwardToken": "f"})
            if not body["startFromHead"] and body.get("nextToken", "").startswith("b/") and \
                    body["nextToken"] != "b/end":
                n = int(body["nextToken"].split("/")[1])
                if n < self.backward_empty_pages:
                    return httpx.Response(200, json={"events": [], "nextBackwardToken": f"b/{n + 1}"})
            limit = body.get("limit", 10000)
            page = evs[:limit] if body["startFromHead"] else evs[-limit:]
            return httpx.Response(200, json={"events": page, "nextBackwardToken": "b/end", "nextForwardToken": "f"})
        return self._err(400, "InvalidOperationException")


def _ev(ts_ms: int, text: str = "x") -> dict:
    return {"timestamp": ts_ms, "message": base64.b64encode(text.encode()).decode()}


def _now_ms() -> int:
    return int(time.time() * 1000)


@pytest.fixture
def cw():
    return FakeCloudWatch()


def _storage(cw, group="dstack"):
    return CloudWatchLogStorage(group, region="eu-west-1", client=cw.client(), credentials=CREDS)


# ---- file backend -----------------------------------------------------------------------------
def test_file_storage_writes_and_polls(tmp_path):
    st = FileLogStorage(tmp_path)
    now = _now_ms()
    st.write_logs("p", "r", "sub", [_ev(now, "runner line")], [_ev(now + 1, "job 1"), _ev(now + 2, "job 2")])
    job = st.poll_logs("p", "r", "sub")
    assert [base64.b64decode(e.message).decode() for e in job.logs] == ["job 1", "job 2"]
    runner = st.poll_logs("p", "r", "sub", diagnose=True)
    assert [base64.b64decode(e.message).decode() for e in runner.logs] == ["runner line"]
    assert (tmp_path / "projects" / "p" / "logs" / "r" / "sub" / "job.log").exists() or \
        any(tmp_path.rglob("job.log"))


# ---- CloudWatch: start-up -----------------------------------------------------------------------
def test_cloudwatch_init_error_without_credentials(cw):
    with pytest.raises(LogStorageError, match="credentials"):
        CloudWatchLogStorage("dstack", client=cw.client(), credentials=(None, None, None))


def test_cloudwatch_init_error_on_request_failure(cw):
    cw.fail["DescribeLogStreams"] = (500, "ServiceUnavailableException")
    with pytest.raises(LogStorageError, match="ServiceUnavailable"):
        _storage(cw)


def test_cloudwatch_init_error_when_group_missing(cw):
    with pytest.raises(LogStorageError, match="LogGroup 'nope' does not exist"):
        _storage(cw, group="nope")
    assert cw.requests[0] == ("DescribeLogStreams", {"logGroupName": "nope", "limit": 1})


# ---- streams ------------------------------------------------------------------------------------
def test_cloudwatch_creates_new_stream(cw):
    st = _storage(cw)
    st.write_logs("p", "run", "s1", [], [_ev(_now_ms())])
    assert "p/run/s1/job" in cw.groups["dstack"]
    assert [t for t, _ in cw.requests].count("CreateLogStream") == 1


def test_cloudwatch_reuses_existing_stream(cw):
    cw.groups["dstack"]["p/run/s1/job"] = []
    st = _storage(cw)
    st.write_logs("p", "run", "s1", [], [_ev(_now_ms())])
    assert [t for t, _ in cw.requests].count("CreateLogStream") == 0
    assert len(cw.groups["dstack"]["p/run/s1/job"]) == 1


def test_cloudwatch_stream_existence_cached(cw):
    st = _storage(cw)
    for i in range(3):
        st.write_logs("p", "run", "s1", [], [_ev(_now_ms() + i)])
    targets = [t for t, _ in cw.requests]
    assert targets.count("DescribeLogStreams") == 2  # group check + first stream check
    assert targets.count("PutLogEvents") == 3


def test_cloudwatch_recreates_stream_deleted_behind_the_cache(cw):
    st = _storage(cw)
    st.write_logs("p", "run", "s1", [], [_ev(_now_ms())])
    del cw.groups["dstack"]["p/run/s1/job"]  # retention policy removed it
    st.write_logs("p", "run", "s1", [], [_ev(_now_ms() + 5, "again")])
    assert [base64.b64decode(e["message"]).decode() for e in cw.groups["dstack"]["p/run/s1/job"]] == ["again"]


# ---- poll ---------------------------------------------------------------------------------------
def _fill(cw, stream="p/run/s1/job", n=5, base=None):
    base = base or _now_ms() - 10_000
    cw.groups["dstack"][stream] = [_ev(base + i, f"line {i}") for i in range(n)]
    return base


def _texts(logs):
    return [base64.b64decode(e.message).decode() for e in logs.logs]


def test_cloudwatch_poll_non_empty(cw):
    _fill(cw)
    st = _storage(cw)
    logs = st.poll_logs("p", "run", "s1", limit=10)
    assert _texts(logs) == [f"line {i}" for i in range(5)] and logs.next_token is None


def test_cloudwatch_poll_empty_and_missing_stream(cw):
    cw.groups["dstack"]["p/run/s1/job"] = []
    st = _storage(cw)
    assert st.poll_logs("p", "run", "s1").logs == []
    assert st.poll_logs("p", "run", "never-written").logs == []  # ResourceNotFound -> empty


def test_cloudwatch_poll_descending_newest_first(cw):
    _fill(cw)
    st = _storage(cw)
    logs = st.poll_logs("p", "run", "s1", descending=True, limit=2)
    assert _texts(logs) == ["line 4", "line 3"]


def test_cloudwatch_poll_descending_skips_leading_empty_pages(cw):
    _fill(cw)
    cw.backward_empty_pages = 2
    st = _storage(cw)
    logs = st.poll_logs("p", "run", "s1", descending=True, limit=10)
    assert _texts(logs)[0] == "line 4"
    tokens = [b.get("nextToken") for t, b in cw.requests if t == "GetLogEvents"]
    assert tokens == [None, "b/1", "b/2"]


def test_cloudwatch_poll_descending_stops_when_token_repeats(cw):
    cw.groups["dstack"]["p/run/s1/job"] = []

    def stuck(req):
        target = req.headers["x-amz-target"].split(".", 1)[1]
        if target == "GetLogEvents":
            cw.requests.append((target, json.loads(req.content)))
            return httpx.Response(200, json={"events": [], "nextBackwardToken": "same"})
        return cw.handle(req)

    st = CloudWatchLogStorage("dstack", region="eu-west-1", client=httpx.Client(transport=httpx.MockTransport(stuck)),
                              credentials=CREDS)
    assert st.poll_logs("p", "run", "s1", descending=True).logs == []
    assert sum(1 for t, _ in cw.requests if t == "GetLogEvents") == 2


def test_cloudwatch_poll_descending_gives_up_after_max_tries(cw):
    _fill(cw)
    cw.backward_empty_pages = 100
    st = _storage(cw)
    assert st.poll_logs("p", "run", "s1", descending=True).logs == []
    assert sum(1 for t, _ in cw.requests if t == "GetLogEvents") == 1 + CloudWatchLogStorage.MAX_EMPTY_BACKWARD_PAGES


def test_cloudwatch_poll_request_params_ascending(cw):
    _fill(cw)
    st = _storage(cw)
    st.poll_logs("p", "run", "s1", limit=7)
    body = [b for t, b in cw.requests if t == "GetLogEvents"][-1]
    assert body == {"logGroupName": "dstack", "logStreamName": "p/run/s1/job", "limit": 7, "startFromHead": True}


def test_cloudwatch_poll_request_params_descending_diagnose_with_dates(cw):
    cw.groups["dstack"]["p/run/s1/runner"] = []
    st = _storage(cw)
    start = datetime(2026, 1, 1, tzinfo=timezone.utc)
    end = start + timedelta(hours=1)
    st.poll_logs("p", "run", "s1", start_time=start, end_time=end, descending=True, limit=3, diagnose=True)
    body = [b for t, b in cw.requests if t == "GetLogEvents"][0]
    assert body["logStreamName"] == "p/run/s1/runner" and body["startFromHead"] is False
    assert body["startTime"] == int(start.timestamp() * 1000) + 1  # exclusive paging start
    assert body["endTime"] == int(end.timestamp() * 1000)


def test_cloudwatch_poll_other_errors_raise(cw):
    cw.groups["dstack"]["p/run/s1/job"] = []
    st = _storage(cw)
    cw.fail["GetLogEvents"] = (400, "InvalidParameterException")
    with pytest.raises(LogStorageError, match="InvalidParameter"):
        st.poll_logs("p", "run", "s1")


# ---- write --------------------------------------------------------------------------------------
def test_cloudwatch_write_logs_both_streams(cw):
    st = _storage(cw)
    now = _now_ms()
    st.write_logs("p", "run", "s1", [_ev(now, "r")], [_ev(now, "j1"), _ev(now + 1, "j2")])
    g = cw.groups["dstack"]
    assert len(g["p/run/s1/runner"]) == 1 and len(g["p/run/s1/job"]) == 2


def test_cloudwatch_write_other_error_raises(cw):
    st = _storage(cw)
    cw.fail["PutLogEvents"] = (400, "InvalidSequenceTokenException")
    with pytest.raises(LogStorageError, match="InvalidSequenceToken"):
        st.write_logs("p", "run", "s1", [], [_ev(_now_ms())])


def test_cloudwatch_write_sorts_out_of_order_events(cw):
    st = _storage(cw)
    now = _now_ms()
    st.write_logs("p", "run", "s1", [], [_ev(now + 2, "c"), _ev(now, "a"), _ev(now + 1, "b")])
    assert [base64.b64decode(e["message"]).decode() for e in cw.groups["dstack"]["p/run/s1/job"]] == ["a", "b", "c"]


def test_cloudwatch_write_drops_past_and_future_events(cw):
    st = _storage(cw)
    now = _now_ms()
    st.write_logs("p", "run", "s1", [], [_ev(now - 15 * 24 * 3600 * 1000, "ancient"), _ev(now, "now"),
                                         _ev(now + 3 * 3600 * 1000, "future")])
    assert [base64.b64decode(e["message"]).decode() for e in cw.groups["dstack"]["p/run/s1/job"]] == ["now"]


def test_cloudwatch_batches_by_size(cw):
    st = _storage(cw)
    now = _now_ms()
    big = "y" * 200_000  # under the 256 KiB per-message cap; five fit in a 1 MiB batch
    events = [{"timestamp": now + i, "message": big} for i in range(12)]
    st.write_logs("p", "run", "s1", [], events)
    puts = [b for t, b in cw.requests if t == "PutLogEvents"]
    assert len(puts) == 3 and [len(p["logEvents"]) for p in puts] == [5, 5, 2]


def test_cloudwatch_batches_by_count(cw):
    st = _storage(cw)
    now = _now_ms()
    st.write_logs("p", "run", "s1", [], [_ev(now + i // 100) for i in range(25_000)])
    puts = [b for t, b in cw.requests if t == "PutLogEvents"]
    assert [len(p["logEvents"]) for p in puts] == [10000, 10000, 5000]


def test_cloudwatch_batches_by_time_span(cw):
    st = _storage(cw)
    now = _now_ms()
    day = 24 * 3600 * 1000
    st.write_logs("p", "run", "s1", [], [_ev(now - 3 * day), _ev(now - 2 * day - 1), _ev(now - day), _ev(now)])
    puts = [[e["timestamp"] for e in b["logEvents"]] for t, b in cw.requests if t == "PutLogEvents"]
    assert all(p[-1] - p[0] <= day for p in puts) and sum(len(p) for p in puts) == 4 and len(puts) >= 2


def test_cloudwatch_skips_oversized_message(cw):
    st = _storage(cw)
    now = _now_ms()
    st.write_logs("p", "run", "s1", [], [{"timestamp": now, "message": "z" * 300_000}, _ev(now + 1, "ok")])
    assert [base64.b64decode(e["message"]).decode() for e in cw.groups["dstack"]["p/run/s1/job"]] == ["ok"]
