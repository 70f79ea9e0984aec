"""xGMI-topology-aware GPU placement on a host (MI355X addition; no reference counterpart).

The reference hands out GPUs by resource id in discovery order (``runner/internal/shim/
resources.go:63-94``).  On an 8×MI355X node every GPU pair has a direct xGMI link, but on partial
or mixed topologies (and on hosts where one link is down) the set of GPUs given to a multi-GPU
job decides whether RCCL rings run over xGMI or fall back to PCIe.  ``pick_gpus`` chooses, among
the free GPUs, a set that maximises direct xGMI links (then NUMA locality); the same greedy runs
in the shim (``native/common/amdgpu.cpp: pick_gpus_xgmi``) for count-only requests.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence

from dstack_amd.core.models.instances import HostTopology


def _linked(xgmi: Sequence[Sequence[int]], a: int, b: int) -> bool:
    return a < len(xgmi) and b < len(xgmi[a]) and xgmi[a][b] > 0


def pick_gpus(topology: Optional[HostTopology], free: List[int], count: int) -> Optional[List[int]]:
    if count <= 0:
        return []
    if len(free) < count:
        return None
    if len(free) == count or topology is None or not topology.xgmi:
        return sorted(free)[:count]
    xgmi, numa = topology.xgmi, topology.numa
    best, best_score = None, -1
    for seed in free:
        sel = [seed]
        while len(sel) < count:
            cand = max(
                (c for c in free if c not in sel),
                key=lambda c: (sum(4 for x in sel if _linked(xgmi, c, x)) + (1 if numa.get(c) == numa.get(seed) else 0),
                               -c),
            )
            sel.append(cand)
        score = sum(4 for a in sel for b in sel if a != b and _linked(xgmi, a, b))
        score += sum(1 for a in sel if numa.get(a) == numa.get(seed))
        if score > best_score:
            best, best_score = sorted(sel), score
    return best


def busy_set(busy_gpus: str) -> List[int]:
    return [int(x) for x in (busy_gpus or "").split(",") if x != ""]


def block_gpu_groups(topology: HostTopology, total_blocks: int) -> List[List[int]]:
    """Partition a host's GPUs into ``total_blocks`` equal groups that are each as
    xGMI-connected as possible (e.g. 2×4 or 4×2 on an 8-GPU node)."""
    n = len(topology.gpus)
    if total_blocks <= 1 or n == 0:
        return [list(range(n))]
    per = n // total_blocks
    remaining = list(range(n))
    groups = []
    for _ in range(total_blocks):
        g = pick_gpus(topology, remaining, per) or remaining[:per]
        groups.append(g)
        remaining = [x for x in remaining if x not in g]
    return groups


def describe(topology: Optional[HostTopology]) -> Dict[str, object]:
    if topology is None:
        return {}
    n = len(topology.gpus)
    links = sum(1 for a in range(n) for b in range(n) if a != b and _linked(topology.xgmi, a, b)) // 2
    full = n * (n - 1) // 2
    return {"gpus": n, "xgmi_links": links, "fully_connected": n > 1 and links == full}
