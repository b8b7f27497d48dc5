"""Event-level readers: group records by key and fold each raw feature with its monoid aggregator.

Reference: ``AggregatedReader`` / ``AggregateDataReader`` / ``ConditionalDataReader``
(``readers/.../DataReader.scala:206-366``), ``AggregateParams`` / ``ConditionalParams`` (``:279``, ``:351-368``)
and the per-feature event filter ``GenericFeatureAggregator.filterByDateWithCutoff``
(``features/.../aggregators/FeatureAggregator.scala:48-130``). SURVEY.md K32 / C14.

Columnar design: records are sorted once by key (the shuffle of the reference becomes one
``argsort``), each raw feature's extracted values and the event timestamps become flat arrays, the
cutoff / window predicate is evaluated for all events at once, and numeric monoids (sum, max, min,
mean, logical-or) are segmented reductions over the sorted key runs (``torch.scatter_reduce`` on the
engine device). Text / list / map monoids fold per key on the host.
"""
from __future__ import annotations

import random
from collections import OrderedDict
from dataclasses import dataclass
from typing import Any, Callable, List, Optional, Sequence

import numpy as np
import torch

from ..config import default_device
from ..data.columns import NumericColumn, column_from_values
from ..data.dataset import Dataset
from ..features import aggregators as A
from ..features import types as T
from ..features.aggregators import CutOffTime, Event
from .base import DataReader

DAY_MS = 86_400_000


@dataclass
class AggregateParams:
    timestamp_fn: Optional[Callable[[Any], int]] = None
    cutoff_time: CutOffTime = CutOffTime.no_cutoff()


class TimeStampToKeep:
    Min, Max, Random = "Min", "Max", "Random"


@dataclass
class ConditionalParams:
    timestamp_fn: Callable[[Any], int]
    target_condition: Callable[[Any], bool]
    response_window_ms: Optional[int] = 7 * DAY_MS
    predictor_window_ms: Optional[int] = 7 * DAY_MS
    timestamp_to_keep: str = TimeStampToKeep.Random
    cutoff_time_fn: Optional[Callable[[str, Sequence[Any]], CutOffTime]] = None
    drop_if_target_condition_not_met: bool = False
    seed: Optional[int] = None


_NUMERIC = {"SumNumeric": "sum", "MaxNumeric": "amax", "MinNumeric": "amin", "MeanNumeric": "mean",
            "LogicalOr": "amax"}


def _event_mask(dates: np.ndarray, cutoff_ms: np.ndarray, is_response: bool, window: Optional[int]) -> np.ndarray:
    """Vectorized ``filterByDateWithCutoff``; ``cutoff_ms`` is per event (NaN = no cutoff)."""
    no = np.isnan(cutoff_ms)
    c = np.where(no, 0.0, cutoff_ms)
    d = dates.astype(np.float64)
    if window is None:
        m = d >= c if is_response else d < c
    elif is_response:
        m = (d >= c) & (d <= c + window)
    else:
        m = (d < c) & (d >= c - window)
    return m | no


class _GroupedReader(DataReader):
    """Shared machinery: read records from a source reader, sort by key, aggregate per feature."""

    def __init__(self, source: DataReader, key: Callable[[Any], Any], device=None):
        super().__init__(key, device or source.device)
        self.source = source
        self.distributed = False     # see distribute()

    def distribute(self, on: bool = True) -> "_GroupedReader":
        """Row-sharded reading under a process group: every rank takes every ``world``-th record of the
        source, the records are shuffled by key to the rank that owns the key (``parallel.dist.
        shuffle_by_key``, an all-to-all over RCCL / gloo) and each rank aggregates its own keys. The result
        is this rank's row shard (``Dataset.sharded``), so the workflow then fits data-parallel."""
        self.distributed = on
        return self

    def _records(self, params) -> List[Any]:
        recs = self.source.read_records(params)
        if recs is None:
            frame = self.source.read_frame(params)
            if frame is None:
                raise ValueError("aggregate readers need record or frame input")
            recs = frame.to_dict("records")
        return list(recs)

    def _cutoffs(self, keys_sorted, starts, ends, recs_sorted, params) -> tuple:
        raise NotImplementedError

    def generate_dataset(self, raw_features: Sequence, params=None) -> Dataset:
        from ..parallel import dist as D
        recs = self._records(params)
        shard = self.distributed and D.world() > 1
        if shard:
            # records travel with their source index: after the key shuffle they are put back in source
            # order, so the stable key sort below orders each key's records as one process would (the
            # order-dependent aggregators -- ConcatText, ConcatList, UnionConcatTextMap -- then agree)
            mine = [(i, recs[i]) for i in range(D.rank(), len(recs), D.world())]
            pairs = D.shuffle_by_key(mine, lambda p: str(self.key_fn(p[1])))
            pairs.sort(key=lambda p: p[0])
            recs = [r for _, r in pairs]
        dev = self.device or default_device()
        n = len(recs)
        keys = np.asarray([str(self.key_fn(r)) for r in recs], dtype=object)
        order = np.argsort(keys, kind="stable")
        keys_s = keys[order]
        recs_s = [recs[i] for i in order]
        if n:
            brk = np.nonzero(keys_s[1:] != keys_s[:-1])[0] + 1
            starts = np.concatenate([[0], brk])
            ends = np.concatenate([brk, [n]])
        else:
            starts = ends = np.zeros(0, np.int64)
        group_keys = keys_s[starts] if n else np.zeros(0, dtype=object)
        ts, cutoff_per_group, windows, keep_groups = self._cutoffs(keys_s, starts, ends, recs_s, params)
        seg = np.repeat(np.arange(len(starts)), ends - starts)
        cutoff_ev = cutoff_per_group[seg] if len(seg) else np.zeros(0)
        cols = OrderedDict()
        for f in raw_features:
            st = f.origin_stage
            agg = st.aggregator or A.default_aggregator(f.wtype)
            # the generator stage's response flag selects the event window (FeatureAggregator.extract: the stage
            # builds its aggregator with outputIsResponse), so a predictor copy of a response feature aggregates as
            # the response does
            resp = bool(getattr(st, "output_is_response", f.is_response))
            win = st.aggregate_window if st.aggregate_window is not None else windows[1 if resp else 0]
            mask = _event_mask(ts, cutoff_ev, resp, win) if n else np.zeros(0, bool)
            vals = [st.extract(r) for r in recs_s]
            out = self._aggregate(agg, vals, mask, seg, len(starts), resp, ts, dev, f.wtype)
            if isinstance(out, NumericColumn):          # device-side numeric monoid
                if len(keep_groups) != len(starts) or np.any(np.asarray(keep_groups) != np.arange(len(starts))):
                    out = out.take(torch.as_tensor(np.asarray(keep_groups, np.int64), device=dev))
                if not f.wtype.nullable and not bool(out.valid.all()):
                    raise T.NonNullableEmptyException(f"{f.wtype.__name__} cannot contain empty values")
                cols[f.name] = out
            else:
                out = [out[g] for g in keep_groups]
                cols[f.name] = column_from_values(f.wtype, out, dev)
        keys_out = np.asarray([group_keys[g] for g in keep_groups], dtype=object)
        if not shard:
            return Dataset(cols, keys_out, len(keep_groups))
        # global row ids: this rank's keys follow the keys of the lower ranks
        counts = D.all_gather_object(len(keep_groups))
        base = sum(counts[:D.rank()])
        ds = Dataset(cols, keys_out, len(keep_groups),
                     torch.arange(base, base + len(keep_groups), device=dev))
        ds.sharded = True
        return ds

    @staticmethod
    def _aggregate(agg, vals, mask, seg, G, is_response, ts, dev=None, wtype=None):
        """One feature's per-key monoid. Numeric monoids (sum / max / min / mean / logical or) are
        segmented reductions over the key runs on the engine device and come back as a device
        ``NumericColumn`` (the K32 path: no per-key host values); the other monoids fold each key's
        events on the host and return a list of values."""
        red = _NUMERIC.get(agg.name)
        if red is not None and all(v is None or isinstance(v, (int, float, bool, np.number)) for v in vals):
            dev = torch.device("cpu") if dev is None else torch.device(dev)
            ok = np.asarray([v is not None for v in vals], bool) & mask
            x = torch.as_tensor(np.asarray([float(v) if v is not None else 0.0 for v in vals], np.float64), device=dev)
            idx = torch.as_tensor(seg, dtype=torch.int64, device=dev)
            okt = torch.as_tensor(ok, device=dev)
            cnt = torch.zeros(G, dtype=torch.float64, device=dev).index_add_(0, idx, okt.to(torch.float64))
            if red in ("sum", "mean"):
                s = torch.zeros(G, dtype=torch.float64, device=dev).index_add_(
                    0, idx, torch.where(okt, x, torch.zeros_like(x)))
                r = s / cnt.clamp_min(1) if red == "mean" else s
            else:
                fill = -np.inf if red == "amax" else np.inf
                r = torch.full((G,), fill, dtype=torch.float64, device=dev).scatter_reduce(
                    0, idx, torch.where(okt, x, torch.full_like(x, fill)), reduce=red, include_self=True)
            valid = cnt > 0
            if wtype is None:                       # list form (callers outside the reader)
                rl, cl = r.tolist(), cnt.tolist()
                if agg.name == "LogicalOr":
                    return [None if cl[g] == 0 else bool(rl[g]) for g in range(G)]
                return [None if cl[g] == 0 else rl[g] for g in range(G)]
            kind = getattr(wtype, "dtype", "float64")
            r = torch.where(valid, r, torch.zeros_like(r))
            vt = r != 0 if kind == "bool" else (r.to(torch.int64) if kind == "int64" else r)
            return NumericColumn(wtype, vt, valid)
        out = []
        bounds = np.searchsorted(seg, np.arange(G + 1)) if len(seg) else np.zeros(G + 1, np.int64)
        for g in range(G):
            a, b = int(bounds[g]), int(bounds[g + 1])
            evs = [Event(int(ts[i]), vals[i], is_response) for i in range(a, b) if mask[i]]
            out.append(agg.aggregate(evs))
        return out


class AggregateReader(_GroupedReader):
    """``DataReaders.Aggregate``: one row per key, events before the cutoff for predictors and at/after it
    for responses."""

    def __init__(self, source: DataReader, key: Callable[[Any], Any], aggregate_params: Optional[AggregateParams] = None,
                 device=None):
        super().__init__(source, key, device)
        self.params = aggregate_params or AggregateParams()

    def _cutoffs(self, keys_s, starts, ends, recs_s, params):
        fn = self.params.timestamp_fn
        ts = np.asarray([int(fn(r)) if fn is not None else 0 for r in recs_s], np.int64)
        c = self.params.cutoff_time.time_ms
        cut = np.full(len(starts), np.nan if c is None else float(c))
        return ts, cut, (None, None), list(range(len(starts)))


class ConditionalReader(_GroupedReader):
    """``DataReaders.Conditional``: the cutoff of each key is the time of a record meeting the target
    condition; predictors use ``predictor_window_ms`` before it, responses ``response_window_ms`` after."""

    def __init__(self, source: DataReader, key: Callable[[Any], Any], conditional_params: ConditionalParams,
                 device=None):
        super().__init__(source, key, device)
        self.params = conditional_params

    def _cutoffs(self, keys_s, starts, ends, recs_s, params):
        p = self.params
        ts = np.asarray([int(p.timestamp_fn(r)) for r in recs_s], np.int64)
        rng = random.Random(p.seed)
        cut = np.zeros(len(starts))
        keep = []
        import time as _time
        for g, (a, b) in enumerate(zip(starts, ends)):
            group = recs_s[a:b]
            targets = [int(ts[a + i]) for i, r in enumerate(group) if p.target_condition(r)]
            if not targets and p.drop_if_target_condition_not_met:
                continue
            keep.append(g)
            if p.cutoff_time_fn is not None:
                c = p.cutoff_time_fn(str(keys_s[a]), group).time_ms
                cut[g] = np.nan if c is None else float(c)
            elif not targets:
                cut[g] = float(int(_time.time() * 1000))
            elif p.timestamp_to_keep == TimeStampToKeep.Min:
                cut[g] = float(min(targets))
            elif p.timestamp_to_keep == TimeStampToKeep.Max:
                cut[g] = float(max(targets))
            else:
                cut[g] = float(targets[rng.randrange(len(targets))])
        return ts, cut, (p.predictor_window_ms, p.response_window_ms), keep
