"""In-process locksets for the control plane (reference: ``S/services/locking.py:13-81``,
``contributing/LOCKING.md``).

With SQLite the server is a single process, so every background task claims the rows it processes
by adding their ids to a named in-memory lockset; rows already in the set are skipped by other
workers.  ``advisory_lock`` serialises whole operations (e.g. run-name allocation per project).
"""

from __future__ import annotations

import contextlib
import threading
import time
from collections import defaultdict
from typing import Dict, Hashable, Iterable, Iterator, List, Set


class Lockset:
    def __init__(self):
        self._lock = threading.Lock()
        self._items: Set[Hashable] = set()

    def try_add_many(self, keys: Iterable[Hashable]) -> List[Hashable]:
        """Claim the keys not held by anyone; returns the ones claimed."""
        got = []
        with self._lock:
            for k in keys:
                if k not in self._items:
                    self._items.add(k)
                    got.append(k)
        return got

    def add_all_or_nothing(self, keys: Iterable[Hashable]) -> bool:
        keys = list(keys)
        with self._lock:
            if any(k in self._items for k in keys):
                return False
            self._items.update(keys)
            return True

    def remove_many(self, keys: Iterable[Hashable]):
        with self._lock:
            for k in keys:
                self._items.discard(k)

    def __contains__(self, k) -> bool:
        with self._lock:
            return k in self._items

    @contextlib.contextmanager
    def hold(self, keys: Iterable[Hashable], timeout: float = 30.0) -> Iterator[None]:
        """Block until all keys are free, hold them for the duration of the block."""
        keys = list(keys)
        deadline = time.monotonic() + timeout
        while not self.add_all_or_nothing(keys):
            if time.monotonic() > deadline:
                raise TimeoutError(f"timed out waiting for locks {keys}")
            time.sleep(0.005)
        try:
            yield
        finally:
            self.remove_many(keys)


class ResourceLocker:
    def __init__(self):
        self._locksets: Dict[str, Lockset] = defaultdict(Lockset)
        self._named: Dict[str, threading.RLock] = defaultdict(threading.RLock)
        self._guard = threading.Lock()

    def get_lockset(self, namespace: str) -> Lockset:
        with self._guard:
            return self._locksets[namespace]

    @contextlib.contextmanager
    def advisory_lock(self, name: str) -> Iterator[None]:
        with self._guard:
            lk = self._named[name]
        with lk:
            yield


_locker = ResourceLocker()


def get_locker() -> ResourceLocker:
    return _locker


def lockset(namespace: str) -> Lockset:
    return _locker.get_lockset(namespace)
