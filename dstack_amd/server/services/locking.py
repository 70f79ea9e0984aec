"""Locking for the control plane (reference: ``S/services/locking.py:13-81``,
``contributing/LOCKING.md``).

* In-process locksets: every background task claims the rows it processes by adding their ids to
  a named lockset; rows already in the set are skipped by the server's other worker threads.
* Postgres (several server replicas on one database): on top of the lockset, the row itself is
  claimed inside the processing transaction with ``SELECT ... FOR UPDATE SKIP LOCKED``
  (``claim_row``) so another replica skips it, and named operations take a transaction-scoped
  ``pg_advisory_xact_lock`` (``db_advisory_lock``).  With SQLite (one server process) both reduce
  to the in-process primitives.
"""

from __future__ import annotations

import contextlib
import hashlib
import threading
import time
from collections import defaultdict
from typing import Dict, Hashable, Iterable, Iterator, List, Optional, Set

from sqlalchemy import select, text
from sqlalchemy.orm import Session


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
        """Block until all keys are free, hold them for the duration of the block; a wait longer
        than ``timeout`` raises ``ResourceBusyError`` (HTTP 409: retry), not a bare 500."""
        from dstack_amd.core.errors import ResourceBusyError

        keys = list(keys)
        deadline = time.monotonic() + timeout
        while not self.add_all_or_nothing(keys):
            if time.monotonic() > deadline:
                raise ResourceBusyError(f"Resource is being processed ({len(keys)} lock(s) busy), retry")
            time.sleep(0.005)
        try:
            yield
        finally:
            self.remove_many(keys)


def release_at_transaction_end(s: Session, ls: Lockset, keys: Iterable[Hashable]):
    """Keep ``keys`` (already held in ``ls``) until ``s``'s transaction commits or rolls back.

    A status change made under an in-process lock must be committed before the lock is released:
    released at flush time, another thread can re-read the still-committed old row and write its
    own transition over the change when it commits after it."""
    keys = list(keys)
    from sqlalchemy import event

    released = []

    def _release(_session):
        if not released:  # whichever of the two events comes first; a later one must not
            released.append(True)  # release keys another thread has claimed since
            ls.remove_many(keys)

    event.listen(s, "after_commit", _release, once=True)
    event.listen(s, "after_rollback", _release, once=True)


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


def _is_postgres(s: Session) -> bool:
    return s.get_bind().dialect.name == "postgresql"


def claim_row_stmt(model, row_id):
    """The row-claim query: the row's id if no other transaction holds it, else no row."""
    return select(model.id).where(model.id == row_id).with_for_update(skip_locked=True)


def claim_row(s: Session, model, row_id) -> bool:
    """Claim ``row_id`` of ``model`` for the rest of ``s``'s transaction.  Postgres: row lock with
    SKIP LOCKED (False = another replica is processing it); SQLite: always True (the in-process
    lockset already excluded the server's other threads)."""
    if not _is_postgres(s):
        return True
    return s.execute(claim_row_stmt(model, row_id)).scalar_one_or_none() is not None


def advisory_key(name: str) -> int:
    """Stable signed 64-bit key for ``pg_advisory_*`` (Python's hash() is salted per process)."""
    return int.from_bytes(hashlib.blake2b(name.encode(), digest_size=8).digest(), "big", signed=True)


ADVISORY_XACT_LOCK_SQL = "SELECT pg_advisory_xact_lock(:k)"


@contextlib.contextmanager
def db_advisory_lock(s: Optional[Session], name: str) -> Iterator[None]:
    """Serialise a named operation across threads (always) and server replicas (Postgres: held
    until ``s``'s transaction ends)."""
    with _locker.advisory_lock(name):
        if s is not None and _is_postgres(s):
            s.execute(text(ADVISORY_XACT_LOCK_SQL), {"k": advisory_key(name)})
        yield
