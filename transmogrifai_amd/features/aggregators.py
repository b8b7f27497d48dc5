"""Monoid aggregators for event-level raw data.

Reference: default aggregator per type (``features/.../aggregators/MonoidAggregatorDefaults.scala:43-123``),
time-window filtering of events (``FeatureAggregator.scala:48-130``) and ``CutOffTime``
(``CutOffTime.scala:40-72``). Aggregate readers group events by key and fold them with these
monoids; numeric reductions over many keys run as segmented reductions on device
(:mod:`transmogrifai_amd.readers.aggregate`).
"""
from __future__ import annotations

import datetime as _dt
import math
from dataclasses import dataclass
from typing import Any, Callable, Optional

from . import types as T


@dataclass
class Event:
    date: int
    value: Any
    is_response: bool = False


class MonoidAggregator:
    name = "MonoidAggregator"
    zero: Any = None

    def prepare(self, event: Event):
        return event.value

    def plus(self, a, b):
        raise NotImplementedError

    def present(self, r):
        return r

    def aggregate(self, events) -> Any:
        acc = self.zero_value()
        for e in events:
            acc = self.plus(acc, self.prepare(e))
        return self.present(acc)

    def zero_value(self):
        import copy
        return copy.copy(self.zero)

    def to_json(self):
        return {"name": self.name}


def _opt(fn):
    def f(a, b):
        if a is None:
            return b
        if b is None:
            return a
        return fn(a, b)
    return f


class SumNumeric(MonoidAggregator):
    name = "SumNumeric"
    plus = staticmethod(_opt(lambda a, b: a + b))


class MaxNumeric(MonoidAggregator):
    name = "MaxNumeric"
    plus = staticmethod(_opt(max))


class MinNumeric(MonoidAggregator):
    name = "MinNumeric"
    plus = staticmethod(_opt(min))


class MeanNumeric(MonoidAggregator):
    name = "MeanNumeric"
    zero = (0.0, 0)

    def prepare(self, e):
        return (0.0, 0) if e.value is None else (float(e.value), 1)

    def plus(self, a, b):
        return (a[0] + b[0], a[1] + b[1])

    def present(self, r):
        return None if r[1] == 0 else r[0] / r[1]


class SumRealNN(SumNumeric):
    """``SumRealNN`` (``aggregators/Numerics.scala:54``): zero 0.0, so a key without events gets 0.0."""
    name = "SumRealNN"
    zero = 0.0


class MaxRealNN(MaxNumeric):
    """``MaxRealNN`` (``Numerics.scala:70``): zero -inf."""
    name = "MaxRealNN"
    zero = float("-inf")


class MinRealNN(MinNumeric):
    """``MinRealNN`` (``Numerics.scala:77``): zero +inf."""
    name = "MinRealNN"
    zero = float("inf")


class MeanRealNN(MeanNumeric):
    """``MeanRealNN`` (``Numerics.scala:103``): 0.0 for a key without events."""
    name = "MeanRealNN"

    def present(self, r):
        return 0.0 if r[1] == 0 else r[0] / r[1]


class LogicalOr(MonoidAggregator):
    name = "LogicalOr"
    plus = staticmethod(_opt(lambda a, b: bool(a) or bool(b)))


class ConcatText(MonoidAggregator):
    name = "ConcatText"

    def __init__(self, separator=","):
        self.separator = separator

    def plus(self, a, b):
        # ConcatTextWithSeparator's monoid: only a missing value is the zero -- an empty string is a value
        if a is None:
            return b
        if b is None:
            return a
        return f"{a}{self.separator}{b}"

    def to_json(self):
        return {"name": self.name, "separator": self.separator}


class ModePickList(MonoidAggregator):
    name = "ModePickList"
    zero = {}

    def prepare(self, e):
        return {} if e.value is None else {e.value: 1}

    def plus(self, a, b):
        out = dict(a)
        for k, v in b.items():
            out[k] = out.get(k, 0) + v
        return out

    def present(self, r):
        if not r:
            return None
        return min(r.items(), key=lambda kv: (-kv[1], kv[0]))[0]


class ConcatList(MonoidAggregator):
    name = "ConcatList"
    zero = []

    def prepare(self, e):
        return list(e.value or [])

    def plus(self, a, b):
        return list(a) + list(b)


class UnionSet(MonoidAggregator):
    name = "UnionSet"
    zero = frozenset()

    def prepare(self, e):
        return frozenset(e.value or ())

    def plus(self, a, b):
        return frozenset(a) | frozenset(b)


class GeolocationMidpoint(MonoidAggregator):
    """Geographic midpoint (``aggregators/Geolocation.scala:43-138``; the monoid of :mod:`.geo`: WGS84 point
    sums, count and the accuracy box, the accuracy presented from the box's widest side)."""
    name = "GeolocationMidpoint"
    zero = (0.0,) * 10

    def prepare(self, e):
        from . import geo
        v = e.value
        if not v:
            return (0.0,) * 10
        import torch
        return tuple(geo.prepare(torch.tensor([list(v[:3])], dtype=torch.float64))[0].tolist())

    def plus(self, a, b):
        if a[3] == 0.0:
            return b
        if b[3] == 0.0:
            return a
        return (a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3], min(a[4], b[4]), min(a[5], b[5]),
                min(a[6], b[6]), max(a[7], b[7]), max(a[8], b[8]), max(a[9], b[9]))

    def present(self, r):
        from . import geo
        return geo.present(r)


class UnionMap(MonoidAggregator):
    """Key-union merge with a per-value combine."""
    name = "UnionMap"
    zero = {}

    def __init__(self, combine: Callable[[Any, Any], Any], name=None):
        self.combine = combine
        if name:
            self.name = name

    def prepare(self, e):
        return dict(e.value or {})

    def plus(self, a, b):
        out = dict(a)
        for k, v in b.items():
            out[k] = self.combine(out[k], v) if k in out else v
        return out


class UnionGeolocationMidpointMap(MonoidAggregator):
    """Per-key geographic midpoint (``UnionGeolocationMidpointMap``): each key folds the full midpoint monoid
    (sums, count, accuracy box) and is presented once at the end; keys without a location are dropped."""
    name = "UnionGeolocationMidpointMap"
    zero = {}
    _g = GeolocationMidpoint()

    def prepare(self, e):
        return {k: self._g.prepare(Event(0, v)) for k, v in (e.value or {}).items()}

    def plus(self, a, b):
        out = dict(a)
        for k, v in b.items():
            out[k] = self._g.plus(out[k], v) if k in out else v
        return out

    def present(self, r):
        return {k: p for k, p in ((k, self._g.present(v)) for k, v in r.items()) if p}


class CombineVector(MonoidAggregator):
    name = "CombineVector"

    def plus(self, a, b):
        import numpy as np
        if a is None or len(a) == 0:
            return b
        if b is None or len(b) == 0:
            return a
        return np.concatenate([a, b])


def default_aggregator(t) -> MonoidAggregator:
    """Default monoid per feature type (``MonoidAggregatorDefaults.scala:43-123``)."""
    if issubclass(t, T.OPVector):
        return CombineVector()
    if issubclass(t, T.Geolocation):
        return GeolocationMidpoint()
    if issubclass(t, T.OPList):
        return ConcatList()
    if issubclass(t, T.Prediction):
        return UnionMap(lambda a, b: (a + b) / 2.0, "UnionMeanPrediction")
    if issubclass(t, T.MultiPickListMap):
        return UnionMap(lambda a, b: frozenset(a) | frozenset(b), "UnionMultiPickListMap")
    if issubclass(t, T.GeolocationMap):
        return UnionGeolocationMidpointMap()
    if issubclass(t, T.BinaryMap):
        return UnionMap(lambda a, b: a or b, "UnionBinaryMap")
    if issubclass(t, T.DateMap):
        return UnionMap(max, "UnionMaxDateMap")
    if issubclass(t, T.PercentMap):
        return UnionMap(lambda a, b: (a + b) / 2.0, "UnionMeanPercentMap")
    if issubclass(t, T.NumericMap):
        return UnionMap(lambda a, b: a + b, "UnionSumMap")
    if issubclass(t, T.OPMap):
        return UnionMap(lambda a, b: f"{a},{b}" if a and b else (a or b), "UnionConcatTextMap")
    if issubclass(t, T.Binary):
        return LogicalOr()
    if issubclass(t, T.Date):
        return MaxNumeric()
    if issubclass(t, T.Percent):
        return MeanNumeric()
    if issubclass(t, T.RealNN):
        return SumRealNN()
    if issubclass(t, T.OPNumeric):
        return SumNumeric()
    if issubclass(t, T.OPSet):
        return UnionSet()
    if issubclass(t, T.PickList):
        return ModePickList()
    if issubclass(t, (T.Text,)):
        sep = " " if t in (T.Text, T.TextArea) else ","
        return ConcatText(sep)
    raise ValueError(f"No default aggregator mapping for feature type {t}")


@dataclass
class CutOffTime:
    """Cutoff for aggregate readers (``aggregators/CutOffTime.scala:40-72``)."""
    ctype: str
    time_ms: Optional[int]

    @staticmethod
    def unix_epoch(ms: int) -> "CutOffTime":
        return CutOffTime("UnixEpoch", max(int(ms), 0))

    @staticmethod
    def days_ago(days: int) -> "CutOffTime":
        now = _dt.datetime.now(_dt.timezone.utc).replace(hour=0, minute=0, second=0, microsecond=0)
        return CutOffTime("DaysAgo", int((now - _dt.timedelta(days=days)).timestamp() * 1000))

    @staticmethod
    def weeks_ago(weeks: int) -> "CutOffTime":
        return CutOffTime("WeeksAgo", CutOffTime.days_ago(7 * weeks).time_ms)

    @staticmethod
    def ddmmyyyy(s: str) -> "CutOffTime":
        d = _dt.datetime.strptime(s, "%d%m%Y").replace(tzinfo=_dt.timezone.utc)
        return CutOffTime("DDMMYYYY", int(d.timestamp() * 1000))

    @staticmethod
    def no_cutoff() -> "CutOffTime":
        return CutOffTime("NoCutoff", None)


def filter_by_date_with_cutoff(date: int, cutoff: CutOffTime, is_response: bool, window: Optional[int]) -> bool:
    """Event selection rule of ``GenericFeatureAggregator.filterByDateWithCutoff``."""
    if cutoff.time_ms is None:
        return True
    c = cutoff.time_ms
    if window is None:
        return date >= c if is_response else date < c
    if is_response:
        return c <= date <= c + window
    return c - window <= date < c


def aggregator_from_json(d) -> Optional[MonoidAggregator]:
    """Rebuild a (default-family) aggregator from its serialized ``{"className", "value": {"name"}}`` form."""
    if not d:
        return None
    name = (d.get("value") or {}).get("name") or d.get("className")
    simple = {c.name: c for c in (SumNumeric, MaxNumeric, MinNumeric, MeanNumeric, SumRealNN, MaxRealNN, MinRealNN,
                                  MeanRealNN, LogicalOr, ModePickList,
                                  ConcatList, UnionSet, GeolocationMidpoint, CombineVector,
                                  UnionGeolocationMidpointMap)}
    if name in simple:
        return simple[name]()
    if name == "ConcatText":
        return ConcatText((d.get("value") or {}).get("separator", ","))
    probe = {"UnionMeanPrediction": T.Prediction, "UnionMultiPickListMap": T.MultiPickListMap,
             "UnionBinaryMap": T.BinaryMap,
             "UnionMaxDateMap": T.DateMap, "UnionMeanPercentMap": T.PercentMap, "UnionSumMap": T.RealMap,
             "UnionConcatTextMap": T.TextMap}
    if name in probe:
        return default_aggregator(probe[name])
    return None
