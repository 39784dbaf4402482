"""xGMI/NUMA-aware preferred allocation for ``amd.com/gpu``.

The kubelet calls ``GetPreferredAllocation(available, must_include, size)``;
we return the subset that keeps a multi-GPU pod on one xGMI island (every pair
directly linked: RCCL rings then run on point-to-point xGMI links, never PCIe),
then on as few NUMA nodes as possible, then lowest indices (stable, so repeated
requests pack GPUs the same way).

On an 8 x MI355X host every pair is xGMI-linked (7 links per GPU), so the
xGMI term only matters for partitioned hosts / partially-populated meshes and
the NUMA term (two sockets x 4 GPUs) decides. The reference has no allocator
(its capacity is a patched constant, kind-gpu-sim.sh:113).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass
from typing import Iterable

EXHAUSTIVE_LIMIT = 20000  # max combinations scored exhaustively


@dataclass(frozen=True)
class DevInfo:
    id: str
    index: int
    numa: int = -1
    node_id: int = -1
    xgmi_peers: frozenset = frozenset()


def _score(devs: list, by_node: dict) -> tuple:
    xgmi = 0
    pairs = 0
    for a, b in itertools.combinations(devs, 2):
        pairs += 1
        if b.node_id in a.xgmi_peers or a.node_id in b.xgmi_peers:
            xgmi += 1
    numas = len({d.numa for d in devs})
    # higher is better: all-pairs xGMI first, then fewer NUMA nodes, then low indices
    return (xgmi == pairs, xgmi, -numas, -sum(d.index for d in devs))


def preferred(available: Iterable[str], must_include: Iterable[str], size: int, devices: dict) -> list:
    """Pick ``size`` device IDs from ``available`` (superset of ``must_include``).

    ``devices`` maps ID -> DevInfo. Unknown IDs are treated as unlinked, NUMA -1.
    Returns IDs sorted by device index (deterministic).
    """
    avail = list(dict.fromkeys(available))
    must = [d for d in dict.fromkeys(must_include) if d in avail]
    if size <= 0:
        return []
    if size > len(avail):
        size = len(avail)
    if len(must) >= size:
        chosen = sorted(must, key=lambda i: (devices.get(i, DevInfo(i, 1 << 30)).index, i))[:size]
        return chosen

    def info(i):
        return devices.get(i, DevInfo(i, 1 << 30))

    rest = [d for d in avail if d not in must]
    need = size - len(must)
    by_node = {}
    ncomb = _ncr(len(rest), need)
    if ncomb <= EXHAUSTIVE_LIMIT:
        best = None
        best_s = None
        for combo in itertools.combinations(rest, need):
            devs = [info(i) for i in (*must, *combo)]
            s = _score(devs, by_node)
            if best_s is None or s > best_s:
                best, best_s = (*must, *combo), s
        chosen = list(best)
    else:
        # greedy: grow from must_include (or the lowest-index device) by best marginal score
        chosen = list(must) or [min(rest, key=lambda i: info(i).index)]
        pool = [d for d in rest if d not in chosen]
        while len(chosen) < size:
            nxt = max(pool, key=lambda c: _score([info(i) for i in (*chosen, c)], by_node))
            chosen.append(nxt)
            pool.remove(nxt)
    return sorted(chosen, key=lambda i: (info(i).index, i))


def _ncr(n: int, r: int) -> int:
    if r < 0 or r > n:
        return 0
    import math

    return math.comb(n, r)
