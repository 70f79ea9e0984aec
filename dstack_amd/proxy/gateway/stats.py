"""Per-service request statistics (reference: ``P/gateway/services/stats.py:40-141``).

Requests land in 1-second frames per host; ``collect()`` aggregates the last 30/60/300 s into
request counts and mean request time.  Two feeds:

* nginx: ``tail`` the ``dstack_stat`` access log (``<unix ts> <host> <status> <request_time>``),
  rotation-aware (inode/size check);
* the built-in data plane records each proxied request directly.
"""

from __future__ import annotations

import os
import threading
import time
from collections import defaultdict, deque
from typing import Deque, Dict, Optional, Tuple

WINDOWS = (30, 60, 300)
LOG_FORMAT = "$msec $host $status $request_time"


class StatsCollector:
    def __init__(self, access_log: Optional[str] = None):
        self.access_log = access_log
        self._frames: Dict[str, Deque[Tuple[int, int, float]]] = defaultdict(deque)  # host -> (sec, n, total_time)
        self._lock = threading.Lock()
        self._pos = 0
        self._inode = None

    def record(self, host: str, request_time: float, ts: Optional[float] = None):
        sec = int(ts if ts is not None else time.time())
        host = host.split(":")[0].lower()
        with self._lock:
            q = self._frames[host]
            if q and q[-1][0] == sec:
                s, n, tot = q[-1]
                q[-1] = (s, n + 1, tot + request_time)
            else:
                q.append((sec, 1, request_time))
            while q and q[0][0] < sec - max(WINDOWS):
                q.popleft()

    def _read_log(self):
        if not self.access_log or not os.path.exists(self.access_log):
            return
        st = os.stat(self.access_log)
        if self._inode != st.st_ino or st.st_size < self._pos:  # rotated or truncated
            self._inode, self._pos = st.st_ino, 0
        with open(self.access_log) as f:
            f.seek(self._pos)
            for line in f:
                if not line.endswith("\n"):
                    break  # partial line: re-read next time
                self._pos += len(line.encode())
                parts = line.split()
                if len(parts) < 4:
                    continue
                try:
                    ts, host, _status, rt = float(parts[0]), parts[1], parts[2], float(parts[3])
                except ValueError:
                    continue
                self.record(host, rt, ts)

    def collect(self) -> Dict[str, Dict[int, Dict[str, float]]]:
        """``{host: {window_s: {"requests": n, "request_time": mean_s}}}``"""
        self._read_log()
        now = int(time.time())
        out: Dict[str, Dict[int, Dict[str, float]]] = {}
        with self._lock:
            for host, q in self._frames.items():
                per = {}
                for w in WINDOWS:
                    n = tot = 0
                    for sec, k, t in q:
                        if sec > now - w:
                            n += k
                            tot += t
                    per[w] = {"requests": n, "request_time": (tot / n) if n else 0.0}
                out[host] = per
        return out
