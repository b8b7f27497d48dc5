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


class LogicalXor(MonoidAggregator):
    """``LogicalXor`` (Numerics.scala:119, 138-143)."""
    name = "LogicalXor"
    plus = staticmethod(_opt(lambda a, b: bool(a) != bool(b)))


class LogicalAnd(MonoidAggregator):
    """``LogicalAnd`` (Numerics.scala:120, 145-150)."""
    name = "LogicalAnd"
    plus = staticmethod(_opt(lambda a, b: bool(a) and bool(b)))


def clip_percent(p: float) -> float:
    """``PercentPrepare.prepareFn``: a percent below 0 counts as 0, above 1 as 1."""
    return 0.0 if p < 0.0 else 1.0 if p > 1.0 else p


class MeanPercent(MeanNumeric):
    """``MeanPercent`` (Numerics.scala:105): the mean of the values clipped to [0, 1]."""
    name = "MeanPercent"

    def prepare(self, e):
        return (0.0, 0) if e.value is None else (clip_percent(float(e.value)), 1)


def concat_text(a: str, b: str, sep: str) -> str:
    """``TextUtils.concat``: l if r is empty, r if l is empty, else l + sep + r."""
    if not a:
        return b
    if not b:
        return a
    return f"{a}{sep}{b}"


class ConcatText(MonoidAggregator):
    name = "ConcatText"

    def __init__(self, separator=","):
        self.separator = separator

    def plus(self, a, b):
        # ConcatTextWithSeparator's monoid (aggregators/Text.scala:50-54): a missing value is the zero, present
        # values join with TextUtils.concat (an empty side contributes nothing, so ("", "") stays a present "")
        if a is None:
            return b
        if b is None:
            return a
        return concat_text(a, b, self.separator)

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


class TimeBasedAggregator(MonoidAggregator):
    """``LastAggregator`` / ``FirstAggregator`` (TimeBasedAggregator.scala:38-75): the value of the latest
    (earliest) event by date -- ties keep the left value for Last and take the right one for First, as the
    reference's ``compareFun``; an empty event value is a value like any other."""

    def __init__(self, is_last: bool = True, name: Optional[str] = None):
        self.is_last = is_last
        self.name = name or ("LastAggregator" if is_last else "FirstAggregator")
        self.zero = (0, None) if is_last else ((1 << 63) - 1, None)

    def prepare(self, e):
        return (int(e.date), e.value)

    def plus(self, a, b):
        if self.is_last:
            return b if a[0] < b[0] else a
        return b if a[0] >= b[0] else a

    def present(self, r):
        return r[1]

    def to_json(self):
        return {"name": self.name, "isLast": self.is_last}


def LastAggregator(name: Optional[str] = None) -> TimeBasedAggregator:
    return TimeBasedAggregator(True, name)


def FirstAggregator(name: Optional[str] = None) -> TimeBasedAggregator:
    return TimeBasedAggregator(False, name)


class MinMaxList(MonoidAggregator):
    """``MinMaxList`` (Lists.scala): the single smallest / largest element of all the lists (``MinDateList``,
    ``MaxDateList``, ``MinDateTimeList``, ``MaxDateTimeList``)."""
    zero = ()

    def __init__(self, is_min: bool, name: str):
        self.is_min, self.name = is_min, name

    def prepare(self, e):
        v = list(e.value or ())
        return (min(v) if self.is_min else max(v),) if v else ()

    def plus(self, a, b):
        v = list(a) + list(b)
        return (min(v) if self.is_min else max(v),) if v else ()

    def present(self, r):
        return list(r)

    def to_json(self):
        return {"name": self.name}


class UnionMeanMap(MonoidAggregator):
    """``UnionMeanDoubleMap`` (Maps.scala:58-74): per-key (sum, count), presented as the mean (0.0 for a key
    seen without values); ``clip`` is the percent variant."""
    zero = {}

    def __init__(self, name: str = "UnionMeanRealMap", clip: bool = False):
        self.name, self.clip = name, clip

    def prepare(self, e):
        f = clip_percent if self.clip else float
        return {k: (f(float(v)), 1) for k, v in (e.value or {}).items() if v is not None}

    def plus(self, a, b):
        out = dict(a)
        for k, (sv, n) in b.items():
            s0, n0 = out.get(k, (0.0, 0))
            out[k] = (s0 + sv, n0 + n)
        return out

    def present(self, r):
        return {k: (sv / n if n else 0.0) for k, (sv, n) in r.items()}

    def to_json(self):
        return {"name": self.name}


class UnionMinMaxMap(UnionMap):
    """``UnionMinMaxNumericMap`` (Maps.scala:106-126): per-key min or max."""

    def __init__(self, is_min: bool, name: str):
        super().__init__(min if is_min else max, name)


class UnionConcatTextMap(UnionMap):
    """``UnionConcatTextMap`` (Maps.scala:132-153): per-key ``TextUtils.concat`` with the type's separator (a
    space for TextMap / TextAreaMap, a comma otherwise)."""

    def __init__(self, separator: str = ",", name: str = "UnionConcatTextMap"):
        self.separator = separator
        super().__init__(lambda a, b: concat_text(a, b, separator), name)

    def to_json(self):
        return {"name": self.name, "separator": self.separator}


class SumVector(MonoidAggregator):
    """``SumVector`` (OPVector.scala): element-wise sum; vectors of different lengths are an error."""
    name = "SumVector"

    def plus(self, a, b):
        import numpy as np
        if a is None or len(a) == 0:
            return b
        if b is None or len(b) == 0:
            return a
        if len(a) != len(b):
            raise ValueError(f"requirement failed: Vectors must have same length: x.length == y.length "
                             f"({len(b)} != {len(a)})")
        return np.asarray(a, np.float64) + np.asarray(b, np.float64)


class CustomMonoidAggregator(MonoidAggregator):
    """``CustomMonoidAggregator``: a user zero and associative function over the raw values."""
    name = "CustomMonoidAggregator"

    def __init__(self, zero, associative_fn):
        self.zero, self.fn = zero, associative_fn

    def plus(self, a, b):
        return self.fn(a, b)


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
        return UnionMeanMap("UnionMeanPrediction")
    if issubclass(t, T.MultiPickListMap):
        return UnionMap(lambda a, b: frozenset(a) | frozenset(b), "UnionMultiPickListMap")
    if issubclass(t, T.GeolocationMap):
        return UnionGeolocationMidpointMap()
    if issubclass(t, T.BinaryMap):
        return UnionMap(lambda a, b: a or b, "UnionBinaryMap")
    if issubclass(t, T.DateMap):
        return UnionMap(max, "UnionMaxDateMap")
    if issubclass(t, T.PercentMap):
        return UnionMeanMap("UnionMeanPercentMap", clip=True)
    if issubclass(t, T.NumericMap):
        return UnionMap(lambda a, b: a + b, "UnionSumMap")
    if issubclass(t, T.OPMap):
        sep = " " if t in (T.TextMap, T.TextAreaMap) else ","
        return UnionConcatTextMap(sep)
    if issubclass(t, T.Binary):
        return LogicalOr()
    if issubclass(t, T.Date):
        return MaxNumeric()
    if issubclass(t, T.Percent):
        return MeanPercent()
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
                                  MeanRealNN, LogicalOr, LogicalXor, LogicalAnd, MeanPercent, ModePickList, SumVector,
                                  ConcatList, UnionSet, GeolocationMidpoint, CombineVector,
                                  UnionGeolocationMidpointMap)}
    if name in simple:
        return simple[name]()
    if name == "ConcatText":
        return ConcatText((d.get("value") or {}).get("separator", ","))
    if name == "UnionConcatTextMap":
        return UnionConcatTextMap((d.get("value") or {}).get("separator", ","))
    if name in ("UnionMeanPrediction", "UnionMeanRealMap", "UnionMeanCurrencyMap", "UnionMeanPercentMap"):
        return UnionMeanMap(name, clip=name == "UnionMeanPercentMap")
    for pre, is_min in (("UnionMin", True), ("UnionMax", False)):
        if name.startswith(pre) and name.endswith("Map"):
            return UnionMinMaxMap(is_min, name)
    if name.startswith("Last") or name.startswith("First"):
        return TimeBasedAggregator(name.startswith("Last"), name)
    if name in ("MinDateList", "MinDateTimeList", "MaxDateList", "MaxDateTimeList"):
        return MinMaxList(name.startswith("Min"), name)
    probe = {"UnionMultiPickListMap": T.MultiPickListMap, "UnionBinaryMap": T.BinaryMap, "UnionSumMap": T.RealMap}
    if name in probe:
        return default_aggregator(probe[name])
    return None
