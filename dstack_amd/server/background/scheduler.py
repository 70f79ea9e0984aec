"""Event-driven interval scheduler for the reconcilers (replaces APScheduler; reference:
``S/background/__init__.py:34-87``).

Every task keeps the reference's fallback interval + jitter, but services also ``wake()`` the
task responsible for the next stage whenever they change state (submitted -> provisioning ->
pulling -> running -> terminating).  A woken task runs immediately on its worker thread, so a job
moves through its stages in the time the work takes instead of in 2-4 s tick quanta — the main
cold-start lever.
"""

from __future__ import annotations

import logging
import random
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

logger = logging.getLogger(__name__)


@dataclass
class _Task:
    name: str
    fn: Callable[[], object]
    interval: float
    jitter: float = 0.0
    workers: int = 1
    event: threading.Event = field(default_factory=threading.Event)
    threads: List[threading.Thread] = field(default_factory=list)
    runs: int = 0
    errors: int = 0
    last_duration: float = 0.0
    echo: bool = False


class Scheduler:
    ECHO_DELAY = 0.15

    def __init__(self):
        self._tasks: Dict[str, _Task] = {}
        self._stop = threading.Event()
        self._started = False

    def add(self, name: str, fn: Callable[[], object], interval: float, jitter: float = 0.0, workers: int = 1):
        self._tasks[name] = _Task(name, fn, interval, jitter, workers)

    def wake(self, *names: str):
        for n in names:
            t = self._tasks.get(n)
            if t is not None:
                t.event.set()

    def _loop(self, t: _Task):
        while not self._stop.is_set():
            start = time.monotonic()
            try:
                more = t.fn()
                t.runs += 1
            except Exception:  # noqa: BLE001 - a reconciler error must not kill the loop
                t.errors += 1
                more = False
                logger.exception("background task %s failed", t.name)
            t.last_duration = time.monotonic() - start
            if more:  # the task processed a full batch: there is probably more work right now
                continue
            if t.echo:
                # a wake() may come from a transaction that commits just after we looked: re-check
                # once shortly after every event-driven run instead of waiting a full interval
                t.echo = False
                wait = self.ECHO_DELAY
            else:
                wait = t.interval + (random.uniform(-t.jitter, t.jitter) if t.jitter else 0.0)
            if t.event.wait(max(0.0, wait)):
                t.echo = True
            t.event.clear()

    def start(self):
        if self._started:
            return
        self._started = True
        for t in self._tasks.values():
            for i in range(t.workers):
                th = threading.Thread(target=self._loop, args=(t,), name=f"bg-{t.name}-{i}", daemon=True)
                th.start()
                t.threads.append(th)

    def shutdown(self, timeout: float = 5.0):
        self._stop.set()
        for t in self._tasks.values():
            t.event.set()
        for t in self._tasks.values():
            for th in t.threads:
                th.join(timeout)

    def stats(self) -> Dict[str, dict]:
        return {n: {"runs": t.runs, "errors": t.errors, "last_duration_s": t.last_duration}
                for n, t in self._tasks.items()}


_scheduler: Optional[Scheduler] = None


def get_scheduler() -> Scheduler:
    global _scheduler
    if _scheduler is None:
        _scheduler = Scheduler()
    return _scheduler


def wake(*names: str):
    """Wake reconcilers (no-op when the scheduler is not running, e.g. in unit tests)."""
    from dstack_amd.server import settings

    if settings.SERVER_EVENT_DRIVEN and _scheduler is not None:
        _scheduler.wake(*names)


def wake_later(delay: float, *names: str):
    """Wake reconcilers after ``delay`` seconds: a pass that finds an agent not ready yet returns at
    once and asks to be run again shortly, instead of sleeping inside its claim (which would stall
    every other row of the batch behind one slow host)."""
    from dstack_amd.server import settings

    if not (settings.SERVER_EVENT_DRIVEN and _scheduler is not None):
        return
    t = threading.Timer(delay, _scheduler.wake, args=names)
    t.daemon = True
    t.start()


# task names
SUBMITTED_JOBS = "process_submitted_jobs"
RUNNING_JOBS = "process_running_jobs"
TERMINATING_JOBS = "process_terminating_jobs"
RUNS = "process_runs"
INSTANCES = "process_instances"
FLEETS = "process_fleets"
VOLUMES = "process_submitted_volumes"
GATEWAYS = "process_submitted_gateways"
GATEWAYS_CONNECTIONS = "process_gateways_connections"
PLACEMENT_GROUPS = "process_placement_groups"
COLLECT_METRICS = "collect_metrics"
DELETE_METRICS = "delete_metrics"
