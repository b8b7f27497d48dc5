"""A fixed, process-wide set of side streams for the concurrent parts of a fit.

Concurrency on one GPU comes from three places: learner lanes (tuning/validators.py), the pipelined boosting
parts (models/trees.py ``_run_parts``) and the tree grower's job groups (models/tree_engine.py). Each used to
create its streams on demand (a torch pool stream per part and lane, a native stream per grower slot), so a
lanes run put a dozen streams on the process's ``GPU_MAX_HW_QUEUES`` = 4 hardware queues. Streams that share
an in-order hardware queue serialise behind each other's barrier packets (every cross-stream join is one), so
the concurrency they were meant to buy turns into head-of-line blocking (docs/ROUND4.md, "lanes").

Here every such user leases from ``TMOG_SIDE_STREAMS`` (default 3) persistent streams created once per device:
with the caller's stream that is one stream per hardware queue. A lease never blocks -- a user that gets fewer
streams than it asked for shares: lanes and boosting parts merge their work, grower groups share a stream --
and none of those choices changes a result (trees and metrics do not depend on the stream layout).

A second set of high-priority streams serves the critical path of a lanes run (``TMOG_LANE_PRIO``): the longest
learner's lane and every stream it leases (its boosting parts, grower groups) run at high queue priority, so
when the lanes' kernels compete for compute units the hardware dispatcher feeds the critical learner first and
the shorter lanes fill the gaps. A lease made from a high-priority stream draws from the high set."""
from __future__ import annotations

import contextlib
import os
import threading
from typing import Dict, List

import torch

_LOCK = threading.Lock()
_POOL: Dict[tuple, List[torch.cuda.Stream]] = {}
_BUSY: Dict[tuple, set] = {}


def n_side() -> int:
    return max(0, int(os.environ.get("TMOG_SIDE_STREAMS", "3")))


def _index(dev) -> int:
    dev = torch.device(dev)
    return dev.index if dev.index is not None else torch.cuda.current_device()


def is_high(stream) -> bool:
    return stream is not None and getattr(stream, "priority", 0) < 0


def lease(dev, n: int, high=None) -> List[torch.cuda.Stream]:
    """Up to ``n`` currently unleased side streams of ``dev`` (possibly none). ``high`` selects the
    high-priority set; by default a caller running on a high-priority stream leases from it."""
    if n <= 0 or torch.device(dev).type != "cuda":
        return []
    i = _index(dev)
    if high is None:
        high = is_high(torch.cuda.current_stream(torch.device("cuda", i)))
    key = (i, bool(high))
    with _LOCK:
        pool = _POOL.get(key)
        if pool is None:
            pool = _POOL[key] = [torch.cuda.Stream(device=torch.device("cuda", i), priority=-1 if high else 0)
                                 for _ in range(n_side())]
            _BUSY[key] = set()
        busy = _BUSY[key]
        got = [k for k in range(len(pool)) if k not in busy][:n]
        busy.update(got)
        return [pool[k] for k in got]


def release(dev, streams: List[torch.cuda.Stream]) -> None:
    if not streams:
        return
    i = _index(dev)
    with _LOCK:
        for key in ((i, False), (i, True)):
            if key not in _POOL:
                continue
            pool, busy = _POOL[key], _BUSY[key]
            for s in streams:
                for k, p in enumerate(pool):
                    if p == s:
                        busy.discard(k)


@contextlib.contextmanager
def leased(dev, n: int, high=None):
    got = lease(dev, n, high)
    try:
        yield got
    finally:
        release(dev, got)


_LANES = {"n": 1}


def set_active_lanes(n: int) -> None:
    """Learner lanes running at once on this process's GPU (tuning/validators.py sets it around a lanes run):
    device-memory budgets taken while lanes run are shared between them (models/trees.py _budget_chunks)."""
    _LANES["n"] = max(1, int(n))


def active_lanes() -> int:
    return _LANES["n"]


def in_use(dev) -> int:
    """Streams of ``dev`` currently leased (tests / diagnostics)."""
    i = _index(dev)
    with _LOCK:
        return len(_BUSY.get((i, False), ())) + len(_BUSY.get((i, True), ()))
