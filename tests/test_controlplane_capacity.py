"""The reference's only like-for-like control-plane numbers: one server replica handles 150 active
jobs with at most 2 minutes of processing latency, and processes 75 submissions per minute
(``src/dstack/_internal/server/background/__init__.py:39-46``).  ``bench_controlplane.py`` drives
the real app (HTTP API, SQLite, event-driven reconcilers) with fake agents that answer after an
SSH-like round trip; this runs it at 150 jobs and checks those bounds."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_150_active_jobs_within_reference_bounds(tmp_path):
    out = tmp_path / "cp.json"
    r = subprocess.run([sys.executable, "bench_controlplane.py", "--jobs", "150", "--hold-s", "8",
                        "--rpc-latency-ms", "10", "--out", str(out)], cwd=REPO, capture_output=True, text=True,
                       timeout=900, env=dict(os.environ, PYTHONPATH=REPO))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["running"] == 150 and d["jobs_left"] == 0
    assert d["submit_to_running_s"]["max"] <= 120  # every job RUNNING within the reference's bound
    assert d["pull_interval_s"]["max"] <= 120  # no running job's state older than 2 minutes
    assert d["processed_per_min"] >= 75  # at least the reference's peak processing rate
