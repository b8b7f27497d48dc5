"""Intra-job parallelism of the model-selector learners across ranks (one rank per GPU).

The reference parallelises *inside* a fit through Spark: every MLlib L-BFGS iteration is a
``treeAggregate`` of the gradient over row partitions and XGBoost4J grows each
tree with ``numWorkers`` Rabit workers (``OpXGBoostClassifier.scala:111``, tracker at
``XGBoostParams.scala:69``; C18). Sharding whole (learner, grid point, fold) jobs over ranks alone
cannot use 8 GPUs when a handful of boosting jobs dominate, so two intra-job modes exist:

* **rows** (linear learners): every rank runs *all* of the learner's jobs on a contiguous 1/R slice of
  the (replicated) training rows; the objective's per-problem sums -- loss, gradient ``X^T R``,
  intercept residual -- are all-reduced once per pass in one fused buffer. The quasi-Newton updates
  then run identically on every rank, so all ranks hold the same coefficients.
* **features** (boosted / single trees): every rank grows every tree of every job on the replicated
  binned matrix but builds histograms and scans splits for its own slice of the features only; per
  tree level one RCCL all-gather of the per-node best splits (a few hundred bytes) over xGMI lets all
  ranks take the same decisions (``ops/csrc/common/tree_grow.hpp``). Histogram traffic never crosses
  the links: at depth 10 a histogram all-reduce would move tens of MB per level, the split exchange
  moves ~40 bytes per node.

:class:`LearnerParallel` is handed to learners through the validator's context (``context["par"]``).
"""
from __future__ import annotations

import ctypes as C
import logging
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import dist as D

log = logging.getLogger(__name__)

_EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64)


class FeatureParallel:
    """Communication context of the feature-parallel tree grower.

    GPU: one RCCL communicator per grower job group (each group runs on its own host thread and HIP
    stream, so each needs its own communicator to keep collective order per group); created once per
    process: rank 0's unique id is broadcast through ``torch.distributed``, every rank joins on its
    current device. CPU: an all-gather callback over a gloo group (the tests' multi-process path)."""

    _comms: Dict[tuple, int] = {}

    def __init__(self, rank: Optional[int] = None, world: Optional[int] = None, group: Optional[D.RankGroup] = None):
        self.group = group
        if group is not None:
            self.rank, self.world = group.rank, group.world
        else:
            self.rank = D.rank() if rank is None else rank
            self.world = D.world() if world is None else world
        self._cpu_group = None
        self._cb = None

    # -- GPU -------------------------------------------------------------------------------------
    def comm_array(self, device: torch.device, n_groups: int):
        from ..ops import _native as N
        lib = N.hip()
        if D.simulated():
            # single-GPU projection of this rank's share (scripts/project_schedule.py): no peers to talk to -- the
            # grower answers the split-record exchange locally (tree_grow_hip.hip tmog_hip_fp_allgather)
            return (C.c_void_p * max(1, n_groups))(*([None] * max(1, n_groups)))
        dev = device.index if device.index is not None else torch.cuda.current_device()
        handles = []
        members = self.group.ranks if self.group is not None else tuple(range(self.world))
        for g in range(n_groups):
            key = (dev, members, self.rank, g)
            h = FeatureParallel._comms.get(key)
            if h is None:
                uid = None
                if self.rank == 0:
                    buf = C.create_string_buffer(256)
                    n = lib.tmog_hip_rccl_unique_id(buf, 256)
                    if n <= 0:
                        raise RuntimeError("ncclGetUniqueId failed")
                    uid = buf.raw[:n]
                # the group's leader (rank 0 of the group) generated it; broadcast inside the group
                uid = D.broadcast_object(uid, members[0], self.group) if self.group is not None \
                    else D.broadcast_object(uid, 0)
                with torch.cuda.device(dev):
                    h = lib.tmog_hip_rccl_comm_init(C.c_char_p(uid), self.world, self.rank)
                if not h:
                    raise RuntimeError("ncclCommInitRank failed for the feature-parallel tree grower")
                FeatureParallel._comms[key] = h
            handles.append(h)
        arr = (C.c_void_p * max(1, n_groups))(*handles)
        return arr

    # -- CPU -------------------------------------------------------------------------------------
    def exchange_fn(self):
        """ctypes callback ``(ctx, group, send, recv, bytes) -> 0`` all-gathering ``bytes`` per rank."""
        import torch.distributed as dist
        if self._cb is not None:
            return self._cb
        if self.group is not None:
            # a rank subgroup: its gloo twin was created collectively with it (dist.partition)
            self._cpu_group = self.group.cpu_pg or self.group.pg
        elif D.is_dist() and dist.get_backend() != "gloo":
            self._cpu_group = dist.new_group(backend="gloo")
        world, grp = self.world, self._cpu_group

        def _exchange(ctx, group, send, recv, nbytes):
            if world <= 1:
                C.memmove(recv, send, int(nbytes))
                return 0
            try:
                src = np.ctypeslib.as_array((C.c_uint8 * int(nbytes)).from_address(send)).copy()
                t = torch.from_numpy(src)
                outs = [torch.empty_like(t) for _ in range(world)]
                dist.all_gather(outs, t, group=grp)
                cat = torch.cat(outs).numpy()
                C.memmove(recv, cat.ctypes.data, int(nbytes) * world)
                return 0
            except Exception as e:     # surfaced by the grower as "feature-parallel exchange failed"
                log.error("feature-parallel exchange failed: %r", e)
                return 1

        self._cb = _EXCHANGE_FN(_exchange)
        return self._cb


class LearnerParallel:
    """What a learner needs to split one batch of jobs over all ranks, or over the ranks of one
    :class:`parallel.dist.RankGroup` (hybrid schedules: each group of ranks runs its own jobs, every job
    spread over the group, parallel/scheduler.py)."""

    def __init__(self, rank: Optional[int] = None, world: Optional[int] = None, group: Optional[D.RankGroup] = None):
        self.group = group
        if group is not None:
            self.rank, self.world = group.rank, group.world
        else:
            self.rank = D.rank() if rank is None else rank
            self.world = D.world() if world is None else world
        self.fp = FeatureParallel(self.rank, self.world, group)

    # -- rows ------------------------------------------------------------------------------------
    def row_slice(self, n: int) -> slice:
        """This rank's contiguous share of ``n`` rows (balanced to +-1 row)."""
        a = (n * self.rank) // self.world
        b = (n * (self.rank + 1)) // self.world
        return slice(a, b)

    def sum(self, *tensors: torch.Tensor) -> List[torch.Tensor]:
        """Element-wise sum over ranks of several tensors in one collective (float64 on the wire)."""
        if self.world <= 1:
            return list(tensors)
        return D.bucketed_all_reduce(list(tensors), "sum", self.group)


def feature_slices(n_multi: int, one_weights: Sequence[float], world: int,
                   force: bool = False) -> Optional[List[Tuple[int, int, int, int]]]:
    """Per-rank ``(mlo, mhi, olo, ohi)`` slices of the grower's multi-bin and one-present-bin feature
    lists: the multi-bin list is cut into near-equal counts (one byte gather + one LDS atomic per row
    each) and the one-present list by cumulative weight (``one_weights`` = present entries per row of
    each column, what its CSR histogram costs). Every rank needs >= 1 multi-bin column (node totals
    are read from the first one), so ``None`` when ``n_multi < world``."""
    if (world <= 1 and not force) or n_multi < max(world, 1):
        return None
    w = np.asarray(one_weights, np.float64)
    n_one = int(w.size)
    out = []
    cw = np.concatenate([[0.0], np.cumsum(w)]) if n_one else np.zeros(1)
    tot = float(cw[-1])
    prev_o = 0
    for r in range(world):
        mlo, mhi = (n_multi * r) // world, (n_multi * (r + 1)) // world
        if r == world - 1:
            ohi = n_one
        elif tot > 0:
            ohi = int(np.searchsorted(cw, tot * (r + 1) / world, side="left"))
            ohi = min(max(ohi, prev_o), n_one)
        else:
            ohi = (n_one * (r + 1)) // world
        out.append((mlo, mhi, prev_o, ohi))
        prev_o = ohi
    return out
