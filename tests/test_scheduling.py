"""Scheduling logic (reference: ``src/tests/_internal/server/services/services/test_autoscalers.py``,
``test_pools.py``, ``background/tasks/test_process_submitted_jobs.py``): autoscalers, xGMI GPU
placement, GPU blocks, request statistics, the event-driven scheduler."""

import threading
import time
from datetime import timedelta

import pytest

from dstack_amd.core.models.instances import GpuDevice, HostTopology
from dstack_amd.server.background.scheduler import Scheduler
from dstack_amd.server.services.services import (
    GPUUtilAutoscaler,
    ManualScaler,
    ReplicaInfo,
    RequestStats,
    RPSAutoscaler,
)
from dstack_amd.server.services.topology import block_gpu_groups, describe, pick_gpus
from dstack_amd.utils.common import get_current_datetime


def _replicas(n, age_s=3600):
    ts = get_current_datetime() - timedelta(seconds=age_s)
    return [ReplicaInfo(active=True, timestamp=ts) for _ in range(n)]


# ---- autoscalers ------------------------------------------------------------------------------
def test_manual_scaler_clips_to_range():
    s = ManualScaler(1, 3)
    assert s.scale([], None) == 1
    assert s.scale(_replicas(5), None) == -2
    assert s.scale(_replicas(2), None) == 0


@pytest.mark.parametrize("rps,active,expected", [(0, 1, 0), (25, 1, 2), (100, 2, 8), (5, 4, -3), (1000, 1, 9)])
def test_rps_autoscaler_target_tracking(rps, active, expected):
    s = RPSAutoscaler(1, 10, target=10, scale_up_delay=0, scale_down_delay=0)
    assert s.scale(_replicas(active), rps) == expected


def test_rps_autoscaler_respects_delays():
    s = RPSAutoscaler(1, 10, target=10, scale_up_delay=300, scale_down_delay=600)
    fresh = _replicas(2, age_s=10)  # changed 10 s ago
    assert s.scale(fresh, 100) == 0  # up-scale waits for the delay
    assert s.scale(fresh, 1) == 0  # down-scale too
    assert s.scale(_replicas(2, age_s=400), 100) == 8
    assert s.scale(_replicas(2, age_s=400), 1) == 0  # down delay is longer
    assert s.scale(_replicas(2, age_s=700), 1) == -1


def test_rps_autoscaler_scale_from_zero_immediately():
    s = RPSAutoscaler(0, 4, target=5, scale_up_delay=300, scale_down_delay=600)
    assert s.scale([], 12) == 3


def test_gpu_util_autoscaler():
    s = GPUUtilAutoscaler(1, 8, target=70, scale_up_delay=0, scale_down_delay=0)
    assert s.scale(_replicas(2), 95.0) == 1  # ceil(2*95/70)=3
    assert s.scale(_replicas(4), 20.0) == -2  # ceil(4*20/70)=2
    assert s.scale(_replicas(8), 99.0) == 0  # capped at max
    assert s.scale(_replicas(2), None) == 0  # no samples: keep within [min, max]


def test_request_stats_windows_and_external():
    st = RequestStats()
    now = time.time()
    for i in range(120):
        st.record("svc", 0.05, now - i * 0.5)  # 2 rps over the last minute
    assert abs(st.rps("svc", 60) - 2.0) < 0.05
    assert abs(st.mean_request_time("svc", 60) - 0.05) < 1e-9
    st.set_external("svc", 3.0, 0.2)  # a gateway saw 3 rps more
    assert abs(st.rps("svc", 60) - 5.0) < 0.05
    st.forget("svc")
    assert st.rps("svc") == 0.0


# ---- xGMI placement ---------------------------------------------------------------------------
def _topo(links):
    n = 8
    x = [[0] * n for _ in range(n)]
    for a, b in links:
        x[a][b] = x[b][a] = 1
    return HostTopology(gpus=[GpuDevice(index=i, name="MI355X") for i in range(n)], xgmi=x,
                        numa={i: i // 4 for i in range(n)})


def test_pick_gpus_fully_connected_quad():
    quads = [(a, b) for q in ((0, 1, 2, 3), (4, 5, 6, 7)) for a in q for b in q if a < b] + [(3, 4)]
    t = _topo(quads)
    got = pick_gpus(t, list(range(8)), 4)
    assert got in ([0, 1, 2, 3], [4, 5, 6, 7])
    assert t.fully_connected(got)
    # with GPU 1 busy the best 3-set is still inside one quad
    got = pick_gpus(t, [0, 2, 3, 4, 5, 6], 3)
    assert t.fully_connected(got)
    assert pick_gpus(t, [0, 1], 3) is None
    assert pick_gpus(None, [5, 2, 7], 2) == [2, 5]


def test_mi355x_full_mesh_blocks():
    full = [(a, b) for a in range(8) for b in range(8) if a < b]
    t = _topo(full)
    assert describe(t) == {"gpus": 8, "xgmi_links": 28, "fully_connected": True}
    groups = block_gpu_groups(t, 4)
    assert len(groups) == 4 and all(len(g) == 2 for g in groups)
    assert sorted(x for g in groups for x in g) == list(range(8))


def test_blocks_follow_partial_topology():
    # two islands: {0,2,4,6} and {1,3,5,7}
    isl = [(a, b) for q in ((0, 2, 4, 6), (1, 3, 5, 7)) for a in q for b in q if a < b]
    t = _topo(isl)
    groups = block_gpu_groups(t, 2)
    assert sorted(map(sorted, groups)) == [[0, 2, 4, 6], [1, 3, 5, 7]]


# ---- event-driven scheduler --------------------------------------------------------------------
def test_scheduler_wake_runs_task_immediately_and_echoes():
    sch = Scheduler()
    calls = []
    ev = threading.Event()

    def task():
        calls.append(time.monotonic())
        if len(calls) >= 3:
            ev.set()
        return False

    sch.add("t", task, interval=30.0)
    sch.start()
    try:
        time.sleep(0.05)  # first run at start
        t0 = time.monotonic()
        sch.wake("t")
        assert ev.wait(2.0), "woken task (+ its echo re-check) did not run"
        # run 2 is the wake, run 3 the echo ~ECHO_DELAY later; both far sooner than the 30 s interval
        assert calls[1] - t0 < 0.5 and calls[2] - calls[1] < 1.0
    finally:
        sch.shutdown()
    assert sch.stats()["t"]["errors"] == 0


def test_scheduler_survives_task_errors():
    sch = Scheduler()
    n = {"c": 0}

    def bad():
        n["c"] += 1
        raise RuntimeError("boom")

    sch.add("bad", bad, interval=0.01)
    sch.start()
    time.sleep(0.2)
    sch.shutdown()
    assert n["c"] > 2 and sch.stats()["bad"]["errors"] == n["c"]
