"""Data-parallel (row-sharded) fitting: the MI355X replacement of Spark's partition-level
``treeAggregate`` / ``fold`` / ``reduceByKey`` statistics (SURVEY.md §2.7 C1-C13, §2.8 "Data parallel").

Layout: with ``world`` ranks (one per GPU, ``torch.distributed`` over RCCL/xGMI, or gloo on the host)
every rank holds a contiguous row shard of the table (:meth:`Dataset.shard`) whose global row ids are
kept, so every seeded per-row decision (hold-out split, folds, down-sampling, bootstrap) is identical
to the single-process run. A workflow fit over a sharded dataset runs inside :func:`scope`; estimator
fits then either

* reduce their partial statistics with one packed collective per fit (``dp_aware`` stages: numeric
  vectorizers, one-hot / set pivots, SanityChecker, the model selector), or
* transparently receive their input columns gathered from every rank (any other estimator: correct
  by construction, just not bandwidth-optimal -- the generic fallback of :func:`gather_column`).

Transformers never communicate: they map local rows to local rows.

Reference reductions replaced here: ``RealVectorizer.scala:84`` / ``IntegralVectorizer.scala:79``
(``SequenceAggregators``), ``OpOneHotVectorizer.scala:97`` (count fold), ``SanityChecker.scala:407,468``
(``colStats``, ``Statistics.corr``), ``SanityChecker.scala:272,280`` (label contingency ``reduceByKey``).
"""
from __future__ import annotations

import threading
from collections import Counter
from contextlib import contextmanager
from typing import Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import dist as D

_STATE = threading.local()
# class names of the estimators whose row-sharded fit fell back to gathering their input columns
# (stages/base.py OpEstimator.fit); empty when every fit reduced its own statistics
GATHER_FALLBACKS: List[str] = []


def active() -> bool:
    """True inside a sharded fit with more than one rank."""
    return bool(getattr(_STATE, "on", False)) and D.world() > 1


@contextmanager
def scope(sharded: bool):
    prev = getattr(_STATE, "on", False)
    _STATE.on = bool(sharded)
    try:
        yield
    finally:
        _STATE.on = prev


@contextmanager
def local_only():
    """Suspend data-parallel reductions (e.g. while fitting on rows already gathered to every rank)."""
    prev = getattr(_STATE, "on", False)
    _STATE.on = False
    try:
        yield
    finally:
        _STATE.on = prev


# ------------------------------------------------------------------------------------ reductions
def sum_(tensors: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    """Element-wise SUM over ranks of several tensors in ONE collective (no-op when not sharded)."""
    if not active():
        return list(tensors)
    return D.bucketed_all_reduce(list(tensors), "sum")


def min_(t: torch.Tensor) -> torch.Tensor:
    return D.all_reduce(t, "min") if active() else t


def max_(t: torch.Tensor) -> torch.Tensor:
    return D.all_reduce(t, "max") if active() else t


def count(n: int) -> int:
    """Global row count."""
    if not active():
        return int(n)
    return int(D.all_reduce(torch.tensor([float(n)], dtype=torch.float64), "sum").item())


def rows(t: torch.Tensor) -> torch.Tensor:
    """All ranks' rows concatenated in rank order (every rank gets the whole tensor)."""
    return D.all_gather_rows(t) if active() else t


def rows_opt(*ts: Optional[torch.Tensor]):
    """:func:`rows` of several optional tensors (``None`` stays ``None``)."""
    return tuple(None if t is None else rows(t) for t in ts)


def merge_counters(counters: Sequence[Counter]) -> List[Counter]:
    """Per-column value counts summed over ranks (one object all-gather for all columns)."""
    if not active():
        return list(counters)
    parts = D.all_gather_object([dict(c) for c in counters])
    out = [Counter() for _ in counters]
    for p in parts:
        for i, c in enumerate(p):
            out[i].update(c)
    return out


def objects(obj) -> list:
    """All ranks' values of a picklable object (single-process: ``[obj]``)."""
    return D.all_gather_object(obj) if active() else [obj]


def unique_values(t: torch.Tensor) -> torch.Tensor:
    """Sorted distinct values over all ranks."""
    u = torch.unique(t)
    if not active():
        return u
    parts = D.all_gather_object(u.cpu().numpy())
    return torch.as_tensor(np.unique(np.concatenate(parts)), dtype=t.dtype, device=t.device)


# ---------------------------------------------------------------------------- generic gathering
def gather_column(col):
    """The whole column (all ranks' rows, rank order) on every rank: the fallback for estimators that
    have no data-parallel reduction of their own."""
    from ..data.columns import (GeoColumn, NumericColumn, ObjectColumn, PredictionColumn, TextColumn,
                                VectorColumn)
    if not active():
        return col
    if isinstance(col, NumericColumn):
        return NumericColumn(col.ftype, D.all_gather_rows(col.values), D.all_gather_rows(col.valid))
    if isinstance(col, TextColumn):
        # shards may have different dictionaries: re-code onto the union vocabulary
        vocabs = D.all_gather_object(list(col.vocab))
        union = sorted(set().union(*[set(v) for v in vocabs]))
        pos = {s: i for i, s in enumerate(union)}
        lut = torch.as_tensor(np.asarray([pos[s] for s in vocabs[D.rank()]] + [-1], np.int64),
                              device=col.codes.device)
        c = col.codes.long()
        local = lut[torch.where(c >= 0, c, torch.full_like(c, lut.numel() - 1))].to(col.codes.dtype)
        return TextColumn(col.ftype, D.all_gather_rows(local), union)
    if isinstance(col, VectorColumn):
        return VectorColumn(D.all_gather_rows(col.values), col.metadata)
    if isinstance(col, GeoColumn):
        return GeoColumn(D.all_gather_rows(col.values), D.all_gather_rows(col.valid))
    if isinstance(col, ObjectColumn):
        parts = D.all_gather_object(col.values)
        return ObjectColumn(col.ftype, np.concatenate(parts) if parts else col.values)
    if isinstance(col, PredictionColumn):
        parts = D.all_gather_object(col.to("cpu"))
        return PredictionColumn.concat(parts).to(col.device)
    parts = D.all_gather_object(col.to("cpu"))
    return type(col).concat(parts).to(col.device)


def gather_dataset(ds, names: Iterable[str]):
    """Dataset restricted to ``names`` with every rank's rows (global row ids kept, not sharded)."""
    from collections import OrderedDict
    from ..data.dataset import Dataset
    cols = OrderedDict((n, gather_column(ds[n])) for n in names)
    rid = D.all_gather_rows(ds.row_ids)
    out = Dataset(cols, None, int(rid.shape[0]), rid)
    out.sharded = False
    return out
