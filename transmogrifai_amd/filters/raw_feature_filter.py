"""RawFeatureFilter: drop raw features whose training / scoring distributions make them unusable.

Reference: ``core/.../op/filters/RawFeatureFilter.scala:90-636`` (exclusion rules, ``generateFilteredRaw``),
``FeatureDistribution.scala`` (fill rate, fill-rate difference / ratio, JS divergence, histograms
``histValues:317-351``), ``Summary.scala:36-66``, ``PreparedFeatures.scala`` (per-type preparation and the
null-indicator / label leakage vector) and ``RawFeatureFilterResults.scala``.

Computation: numeric device columns go through the fused HIP summary + histogram kernels
(``ops/rff.py``); dictionary-coded text columns reduce to per-code counts on the device, and the
per-distinct-value token hashing is done once per vocabulary entry on the host; ragged columns
(lists, sets, maps, vectors, geolocations) use the host row path. The leakage correlation of each
predictor's null indicator with each numeric response is derived from the same sums
(``n, Σy, Σy², Σz, Σyz``) without materializing the indicator matrix.
"""
from __future__ import annotations

import json
import math
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..data.columns import GeoColumn, NumericColumn, ObjectColumn, TextColumn, VectorColumn
from ..data.dataset import Dataset
from ..features import types as T
from ..ops import rff as R
from ..utils.text import hash_terms, tokenize

MAX_BINS = 100_000
MIN_SCORING_ROWS_DEFAULT = 500
MAX_CARDINALITY = 500
TRAINING, SCORING = "Training", "Scoring"

FeatureKey = Tuple[str, Optional[str]]


@dataclass
class Summary:
    min: float = math.inf
    max: float = -math.inf
    sum: float = 0.0
    count: float = 0.0

    def plus(self, o: "Summary") -> "Summary":
        return Summary(min(self.min, o.min), max(self.max, o.max), self.sum + o.sum, self.count + o.count)

    @property
    def is_empty(self) -> bool:
        return self.count == 0 and self.min == math.inf


def _moments_from_sums(c, s1, s2, s3, s4) -> Optional[Dict[str, float]]:
    if c <= 0:
        return {"m0": 0.0, "m1": 0.0, "m2": 0.0, "m3": 0.0, "m4": 0.0}
    m = s1 / c
    m2 = s2 - 2 * m * s1 + c * m * m
    m3 = s3 - 3 * m * s2 + 3 * m * m * s1 - c * m ** 3
    m4 = s4 - 4 * m * s3 + 6 * m * m * s2 - 4 * m ** 3 * s1 + c * m ** 4
    return {"m0": float(c), "m1": float(m), "m2": float(max(m2, 0.0)), "m3": float(m3), "m4": float(max(m4, 0.0))}


@dataclass
class FeatureDistribution:
    """Distribution of one raw feature (or map key) in the training or scoring data."""
    name: str
    key: Optional[str]
    count: int
    nulls: int
    distribution: np.ndarray
    summaryInfo: List[float]
    moments: Optional[Dict[str, float]] = None
    type: str = TRAINING
    # TextStats of the values (FeatureDistribution.scala cardEstimate): {"valueCounts": {value: n}, "lengthCounts":
    # {length: n}}, at most MAX_CARDINALITY + 1 distinct values; in memory only (the reference ignores it in JSON)
    cardEstimate: Optional[Dict[str, Dict]] = None

    @property
    def feature_key(self) -> FeatureKey:
        return (self.name, self.key)

    def fill_rate(self) -> float:
        return 0.0 if self.count == 0 else (self.count - self.nulls) / float(self.count)

    def _check(self, o: "FeatureDistribution"):
        if self.name != o.name or self.key != o.key:
            raise ValueError(f"Name and key must match to compare or combine FeatureDistribution: "
                             f"{self.name}, {self.key} != {o.name}, {o.key}")

    def relative_fill_ratio(self, o: "FeatureDistribution") -> float:
        self._check(o)
        a, b = self.fill_rate(), o.fill_rate()
        small, large = (a, b) if a < b else (b, a)
        return math.inf if small == 0.0 else large / small

    def relative_fill_rate(self, o: "FeatureDistribution") -> float:
        self._check(o)
        return abs(self.fill_rate() - o.fill_rate())

    def js_divergence(self, o: "FeatureDistribution") -> float:
        self._check(o)
        a = np.asarray(self.distribution, np.float64)
        b = np.asarray(o.distribution, np.float64)
        n = min(a.size, b.size)
        a, b = a[:n], b[:n]
        keep = ~((a == 0.0) & (b == 0.0))
        a, b = a[keep], b[keep]
        ta, tb = a.sum(), b.sum()
        if a.size == 0:
            return 0.0
        pa = a / ta if ta > 0 else np.full_like(a, np.nan)
        pb = b / tb if tb > 0 else np.full_like(b, np.nan)
        m = (pa + pb) / 2

        def kl(p, q):
            with np.errstate(divide="ignore", invalid="ignore"):
                t = np.where(p == 0.0, 0.0, p * np.log2(p / q))
            return t
        return float((0.5 * kl(pa, m) + 0.5 * kl(pb, m)).sum())

    def reduce(self, o: "FeatureDistribution") -> "FeatureDistribution":
        self._check(o)
        d = np.asarray(self.distribution, np.float64) + np.asarray(o.distribution, np.float64)
        info = self.summaryInfo if len(self.summaryInfo) > len(o.summaryInfo) else o.summaryInfo
        mom = self.moments
        if self.moments and o.moments:
            mom = _combine_moments(self.moments, o.moments)
        return FeatureDistribution(self.name, self.key, self.count + o.count, self.nulls + o.nulls, d, info,
                                   mom or o.moments, self.type, _card_plus(self.cardEstimate, o.cardEstimate))

    def to_json(self, with_card: bool = False) -> Dict:
        out = {"name": self.name, "key": self.key, "count": int(self.count), "nulls": int(self.nulls),
               "distribution": [float(x) for x in np.asarray(self.distribution).tolist()],
               "summaryInfo": [float(x) for x in self.summaryInfo], "moments": self.moments, "type": self.type}
        if with_card:
            out["cardEstimate"] = self.cardEstimate
        return out

    @staticmethod
    def from_json(d: Dict) -> "FeatureDistribution":
        return FeatureDistribution(d["name"], d.get("key"), int(d["count"]), int(d["nulls"]),
                                   np.asarray(d.get("distribution", []), np.float64), list(d.get("summaryInfo", [])),
                                   d.get("moments"), d.get("type", TRAINING))


def _jstr(x: float) -> str:
    """``Double.toString`` of the JVM (the reference's value keys): plain between 1e-3 and 1e7, else d.dddE+n."""
    x = float(x)
    if x != x or x in (math.inf, -math.inf):
        return "NaN" if x != x else ("Infinity" if x > 0 else "-Infinity")
    if x == 0 or 1e-3 <= abs(x) < 1e7:
        r = repr(x)
        return r if ("." in r or "e" in r) else r + ".0"
    m, e = f"{x:.17e}".split("e")
    m = repr(float(m)).rstrip("0")
    m = m + "0" if m.endswith(".") else m
    return f"{m}E{int(e)}"


def _text_stats(values, weights=None) -> Dict[str, Dict]:
    """``TextStats`` of a value sequence (strings or numbers; optional integer weight per value) with the reference's
    MaxCardinality cap: once more than MAX_CARDINALITY distinct values are seen no new value is added
    (TextStats.monoid)."""
    vc: Dict[str, int] = {}
    lc: Dict[int, int] = {}
    for i, v in enumerate(values):
        w = 1 if weights is None else int(weights[i])
        t = v if isinstance(v, str) else _jstr(v)
        if t in vc:
            vc[t] += w
        elif len(vc) <= MAX_CARDINALITY:
            vc[t] = w
        lc[len(t)] = lc.get(len(t), 0) + w
    return {"valueCounts": vc, "lengthCounts": lc}


def _card_plus(a, b):
    if a is None or b is None:
        return a if b is None else b
    if len(a["valueCounts"]) > MAX_CARDINALITY:
        return a
    if len(b["valueCounts"]) > MAX_CARDINALITY:
        return b
    vc = dict(a["valueCounts"])
    for k, v in b["valueCounts"].items():
        vc[k] = vc.get(k, 0) + v
    lc = dict(a["lengthCounts"])
    for k, v in b["lengthCounts"].items():
        lc[k] = lc.get(k, 0) + v
    return {"valueCounts": vc, "lengthCounts": lc}


def _combine_moments(a, b):
    na, nb = a["m0"], b["m0"]
    n = na + nb
    if n == 0:
        return dict(a)
    d = b["m1"] - a["m1"]
    mean = a["m1"] + d * nb / n
    m2 = a["m2"] + b["m2"] + d * d * na * nb / n
    m3 = (a["m3"] + b["m3"] + d ** 3 * na * nb * (na - nb) / n ** 2 + 3 * d * (na * b["m2"] - nb * a["m2"]) / n)
    m4 = (a["m4"] + b["m4"] + d ** 4 * na * nb * (na * na - na * nb + nb * nb) / n ** 3 +
          6 * d * d * (na * na * b["m2"] + nb * nb * a["m2"]) / n ** 2 + 4 * d * (na * b["m3"] - nb * a["m3"]) / n)
    return {"m0": n, "m1": mean, "m2": m2, "m3": m3, "m4": m4}


@dataclass
class RawFeatureFilterConfig:
    minFill: float
    maxFillDifference: float
    maxFillRatioDiff: float
    maxJSDivergence: float
    maxCorrelation: float
    correlationType: str
    jsDivergenceProtectedFeatures: List[str]
    protectedFeatures: List[str]


@dataclass
class RawFeatureFilterMetrics:
    name: str
    key: Optional[str]
    trainingFillRate: float
    trainingNullLabelAbsoluteCorr: Optional[float]
    scoringFillRate: Optional[float]
    jsDivergence: Optional[float]
    fillRateDiff: Optional[float]
    fillRatioDiff: Optional[float]


@dataclass
class ExclusionReasons:
    name: str
    key: Optional[str]
    trainingUnfilledState: bool
    trainingNullLabelLeaker: bool
    scoringUnfilledState: bool
    jsDivergenceMismatch: bool
    fillRateDiffMismatch: bool
    fillRatioDiffMismatch: bool
    excluded: bool


def _jnum(v):
    if v is None:
        return None
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return str(v)
    return v


@dataclass
class RawFeatureFilterResults:
    rawFeatureFilterConfig: Optional[RawFeatureFilterConfig] = None
    rawFeatureDistributions: List[FeatureDistribution] = field(default_factory=list)
    rawFeatureFilterMetrics: List[RawFeatureFilterMetrics] = field(default_factory=list)
    exclusionReasons: List[ExclusionReasons] = field(default_factory=list)

    def to_json(self) -> Dict:
        return {"rawFeatureFilterConfig": None if self.rawFeatureFilterConfig is None else
                dict(self.rawFeatureFilterConfig.__dict__),
                "rawFeatureDistributions": [d.to_json() for d in self.rawFeatureDistributions],
                "rawFeatureFilterMetrics": [{k: _jnum(v) for k, v in m.__dict__.items()}
                                            for m in self.rawFeatureFilterMetrics],
                "exclusionReasons": [dict(e.__dict__) for e in self.exclusionReasons]}

    @staticmethod
    def from_json(d) -> "RawFeatureFilterResults":
        if isinstance(d, str):
            d = json.loads(d)
        if not d:
            return RawFeatureFilterResults()

        def num(v):
            return float(v) if isinstance(v, str) else v
        cfg = d.get("rawFeatureFilterConfig")
        return RawFeatureFilterResults(
            RawFeatureFilterConfig(**cfg) if cfg else None,
            [FeatureDistribution.from_json(x) for x in d.get("rawFeatureDistributions", [])],
            [RawFeatureFilterMetrics(**{k: num(v) if k not in ("name", "key") else v for k, v in m.items()})
             for m in d.get("rawFeatureFilterMetrics", [])],
            [ExclusionReasons(**e) for e in d.get("exclusionReasons", [])])


@dataclass
class AllFeatureInformation:
    response_summaries: "OrderedDict[FeatureKey, Summary]"
    response_distributions: List[FeatureDistribution]
    predictor_summaries: "OrderedDict[FeatureKey, Summary]"
    predictor_distributions: List[FeatureDistribution]
    correlation_info: Dict[FeatureKey, Dict[FeatureKey, float]]


def _numeric_card(values: torch.Tensor, valid: torch.Tensor) -> Dict[str, Dict]:
    """TextStats of a numeric column: distinct values and their counts in one device pass (``torch.unique``), the
    lowest MAX_CARDINALITY + 1 values kept when there are more."""
    v = values[valid.to(torch.bool)] if valid is not None else values
    u, c = torch.unique(v.to(torch.float64), return_counts=True)
    u, c = u[:MAX_CARDINALITY + 1].cpu().tolist(), c[:MAX_CARDINALITY + 1].cpu().tolist()
    vc = {_jstr(a): int(b) for a, b in zip(u, c)}
    lc: Dict[int, int] = {}
    for a, b in vc.items():
        lc[len(a)] = lc.get(len(a), 0) + b
    return {"valueCounts": vc, "lengthCounts": lc}


# ------------------------------------------------------------------------------------ preparation
class _Prepared:
    """Per feature key: summary, histogram accumulator inputs, null indicator and moments."""

    def __init__(self, n: int):
        self.n = n
        self.summary: "OrderedDict[FeatureKey, Summary]" = OrderedDict()
        self.kind: Dict[FeatureKey, str] = {}          # "num" | "text"
        self.nulls: Dict[FeatureKey, torch.Tensor] = {}  # bool [n] null indicator
        self.power: Dict[FeatureKey, tuple] = {}        # (c, s1, s2, s3, s4) of the moment population
        self.numeric_cols: Dict[FeatureKey, tuple] = {}  # device fast path (values, valid)
        self.values: Dict[FeatureKey, list] = {}        # host path: per row list of values / tokens (None = null)
        self.text_codes: Dict[FeatureKey, tuple] = {}   # (codes tensor, per-vocab token lists)
        self.response_value: Dict[FeatureKey, torch.Tensor] = {}


def _date_value(ms, time_period):
    if time_period is None:
        return float(ms)
    from ..utils.dates import period_values
    return float(period_values(torch.as_tensor([int(ms)], dtype=torch.int64), time_period, raw=True)[0][0])


def _prepare_value(v, ftype, time_period):
    """``PreparedFeatures.prepareFeature`` for one non-map value -> ("num", [floats]) | ("text", [tokens])."""
    if v is None:
        return None
    if issubclass(ftype, T.OPVector):
        arr = np.asarray(v, np.float64).reshape(-1)
        return ("num", arr.tolist())
    if issubclass(ftype, T.Text):
        return ("text", tokenize(v))
    if issubclass(ftype, T.Date):
        return ("num", [_date_value(v, time_period)])
    if issubclass(ftype, T.OPNumeric):
        return ("num", [float(v)])
    if issubclass(ftype, T.Geolocation):
        if not v:
            return None
        return ("num", [float(x) for x in v])
    if issubclass(ftype, T.TextList):
        return ("text", [str(x) for x in v]) if v else None
    if issubclass(ftype, T.DateList):
        return ("num", [_date_value(x, time_period) for x in v]) if v else None
    if issubclass(ftype, T.MultiPickList):
        return ("text", [str(x) for x in v]) if v else None
    raise TypeError(f"Feature type {ftype.__name__} is not supported in RawFeatureFilter")


def _prepare_map(v, ftype, time_period) -> Dict[str, tuple]:
    out = {}
    for k, e in (v or {}).items():
        if e is None:
            continue
        if issubclass(ftype, T.MultiPickListMap):
            out[k] = ("text", [str(x) for x in e])
        elif issubclass(ftype, T.GeolocationMap):
            out[k] = ("num", [float(x) for x in e])
        elif issubclass(ftype, T.DateMap):
            out[k] = ("num", [_date_value(e, time_period)])
        elif isinstance(e, str):
            out[k] = ("text", tokenize(e))
        elif isinstance(e, bool):
            out[k] = ("num", [1.0 if e else 0.0])
        else:
            out[k] = ("num", [float(e)])
    return out


def _prepare(ds: Dataset, features, time_period) -> _Prepared:
    n = len(ds)
    P = _Prepared(n)
    for f in features:
        col = ds[f.name]
        ft = f.wtype
        if isinstance(col, NumericColumn) and not issubclass(ft, T.Date):
            key = (f.name, None)
            P.kind[key] = "num"
            P.numeric_cols[key] = (col.values, col.valid)
            P.nulls[key] = ~col.valid
            if f.is_response:
                P.response_value[key] = torch.where(col.valid, col.values.to(torch.float64),
                                                    torch.zeros_like(col.values, dtype=torch.float64))
            continue
        if isinstance(col, TextColumn) and issubclass(ft, T.Text) and not f.is_response:
            key = (f.name, None)
            P.kind[key] = "text"
            toks = [tokenize(s) for s in col.vocab]
            P.text_codes[key] = (col.codes, toks)
            P.nulls[key] = col.codes < 0
            continue
        vals = col.to_list()
        if issubclass(ft, T.OPMap) and not issubclass(ft, T.Prediction):
            per_key: Dict[str, list] = OrderedDict()
            prepped = [_prepare_map(v, ft, time_period) for v in vals]
            for i, m in enumerate(prepped):
                for k in m:
                    per_key.setdefault(k, [None] * n)[i] = m[k]
            for k in sorted(per_key):
                key = (f.name, k)
                rows = per_key[k]
                kinds = {r[0] for r in rows if r is not None}
                P.kind[key] = "text" if "text" in kinds else "num"
                P.values[key] = [None if r is None else r[1] for r in rows]
            continue
        rows = [_prepare_value(v, ft, time_period) for v in vals]
        key = (f.name, None)
        kinds = {r[0] for r in rows if r is not None}
        P.kind[key] = "text" if "text" in kinds else "num"
        P.values[key] = [None if r is None else r[1] for r in rows]
        if f.is_response:
            P.response_value[key] = torch.tensor([r[1][0] if (r is not None and r[0] == "num" and r[1]) else 0.0
                                                  for r in rows], dtype=torch.float64)
    return P


# ---------------------------------------------------------------------------------------- the filter
class RawFeatureFilter:
    """``RawFeatureFilter`` with the reference defaults (``OpWorkflow.withRawFeatureFilter``, ``:537-552``)."""

    def __init__(self, training_reader=None, scoring_reader=None, bins: int = 100, min_fill_rate: float = 0.001,
                 max_fill_difference: float = 0.90, max_fill_ratio_diff: float = 20.0,
                 max_js_divergence: float = 0.90, max_correlation: float = 0.95, correlation_type: str = "pearson",
                 protected_features: Sequence = (), protected_js_features: Sequence = (),
                 text_bins_formula=None, time_period: Optional[str] = None,
                 min_scoring_rows: int = MIN_SCORING_ROWS_DEFAULT, result_feature_retention_policy: str = "Strict"):
        if not (1 < bins <= MAX_BINS):
            raise ValueError(f"Invalid bin size {bins}, bins must be between 1 and {MAX_BINS}")
        if not 0.0 <= min_fill_rate <= 1.0:
            raise ValueError(f"Invalid minFill size {min_fill_rate}, minFill must be between 0 and 1")
        if not 0.0 <= max_fill_difference <= 1.0:
            raise ValueError("Invalid maxFillDifference, must be between 0 and 1")
        if max_fill_ratio_diff < 0.0:
            raise ValueError("Invalid maxFillRatioDiff, must be greater than 0.0")
        if not 0.0 <= max_js_divergence <= 1.0:
            raise ValueError("Invalid maxJSDivergence, must be between 0 and 1")
        if min_scoring_rows < 0:
            raise ValueError(f"minRowsForScoringSet must be >= 0, but was set to {min_scoring_rows}")
        self.training_reader = training_reader
        self.scoring_reader = scoring_reader
        self.bins = bins
        self.min_fill = min_fill_rate
        self.max_fill_difference = max_fill_difference
        self.max_fill_ratio_diff = max_fill_ratio_diff
        self.max_js_divergence = max_js_divergence
        self.max_correlation = max_correlation
        self.correlation_type = correlation_type.lower()
        self.protected = {n for f in protected_features for n in _raw_names(f)}
        self.js_protected = {n for f in protected_js_features for n in _raw_names(f)}
        self.text_bins_formula = text_bins_formula or (lambda summary, bins: bins)
        self.time_period = time_period
        self.min_scoring_rows = min_scoring_rows
        self.result_feature_retention_policy = result_feature_retention_policy

    # ------------------------------------------------------------------------------------ statistics
    def compute_feature_stats(self, ds: Dataset, features, dist_type: str = TRAINING,
                              info: Optional[AllFeatureInformation] = None) -> AllFeatureInformation:
        responses = [f for f in features if f.is_response and issubclass(f.wtype, T.OPNumeric)]
        predictors = [f for f in features if not f.is_response]
        P = _prepare(ds, responses + predictors, self.time_period)
        resp_keys = [k for k in P.kind if k[0] in {f.name for f in responses}]
        pred_keys = [k for k in P.kind if k[0] in {f.name for f in predictors}]
        n = P.n
        # ---- numeric fast path (one fused device pass for every plain numeric column)
        fast = [k for k in P.numeric_cols]
        label = None
        if resp_keys and resp_keys[0] in P.response_value:
            label = P.response_value[resp_keys[0]]
        stats = {}
        if fast:
            vals = [P.numeric_cols[k][0] for k in fast]
            oks = [P.numeric_cols[k][1] for k in fast]
            lab = None if label is None else label.to(vals[0].device)
            S = R.numeric_summary(vals, oks, lab).cpu().numpy()
            for k, row in zip(fast, S):
                stats[k] = row
        summaries: "OrderedDict[FeatureKey, Summary]" = OrderedDict()
        power: Dict[FeatureKey, tuple] = {}
        for k in P.kind:
            if k in stats:
                row = stats[k]
                s = Summary(row[2], row[3], row[4], row[0]) if row[0] > 0 else Summary()
                summaries[k] = s
                power[k] = (row[0], row[4], row[5], row[6], row[7])
            elif k in P.text_codes:
                codes, toks = P.text_codes[k]
                cnt = _code_counts(codes, len(toks))
                lens = np.array([len(t) for t in toks], np.float64)
                used = cnt > 0
                c = float(cnt.sum())
                s = Summary(float(lens[used].min()), float(lens[used].max()), float((cnt * lens).sum()), c) \
                    if c > 0 else Summary()
                summaries[k] = s
                tl = [np.array([len(x) for x in t], np.float64) for t in toks]
                p = [0.0] * 5
                for w, arr in zip(cnt, tl):
                    if w and arr.size:
                        p[0] += w * arr.size
                        for j in range(1, 5):
                            p[j] += w * float((arr ** j).sum())
                power[k] = tuple(p)
            else:
                rows = P.values[k]
                s = Summary()
                p = [0.0] * 5
                for r in rows:
                    if r is None:
                        continue
                    if P.kind[k] == "text":
                        sz = float(len(r))
                        s = s.plus(Summary(sz, sz, sz, 1.0))
                        arr = np.array([len(x) for x in r], np.float64)
                    else:
                        arr = np.asarray(r, np.float64)
                        if arr.size:
                            s = s.plus(Summary(float(arr.min()), float(arr.max()), float(arr.sum()), float(arr.size)))
                    if arr.size:
                        p[0] += arr.size
                        for j in range(1, 5):
                            p[j] += float((arr ** j).sum())
                summaries[k] = s
                power[k] = tuple(p)
        if info is not None:
            # scoring: bin with the training summaries
            use_sum = OrderedDict(list(info.response_summaries.items()) + list(info.predictor_summaries.items()))
        else:
            use_sum = summaries
        # ---- distributions
        dists: Dict[FeatureKey, FeatureDistribution] = {}
        num_keys = [k for k in fast if k in use_sum]
        if num_keys:
            vals = [P.numeric_cols[k][0] for k in num_keys]
            oks = [P.numeric_cols[k][1] for k in num_keys]
            lo = torch.tensor([use_sum[k].min for k in num_keys], dtype=torch.float64)
            hi = torch.tensor([use_sum[k].max for k in num_keys], dtype=torch.float64)
            H = R.numeric_hist(vals, oks, lo, hi, self.bins).cpu().numpy()
            for k, h in zip(num_keys, H):
                sm = use_sum[k]
                nul = int(stats[k][1])
                if sm.is_empty:
                    info_v, hist = [sm.min, sm.max], np.zeros(0)
                elif sm.min < sm.max:
                    step = (sm.max - sm.min) / (self.bins - 2.0)
                    info_v, hist = [sm.min + step * b for b in range(self.bins)], h
                else:
                    info_v, hist = [sm.min, sm.max, sm.sum, sm.count], h[:2]
                dists[k] = FeatureDistribution(k[0], k[1], n, nul, np.asarray(hist, np.float64), info_v,
                                               _moments_from_sums(*power[k]), dist_type,
                                               _numeric_card(*P.numeric_cols[k]))
        for k in P.kind:
            if k in dists or k not in use_sum:
                continue
            sm = use_sum[k]
            if P.kind[k] == "text":
                nb = int(self.text_bins_formula(sm, self.bins))
                hist = np.zeros(nb)
                if k in P.text_codes:
                    codes, toks = P.text_codes[k]
                    cnt = _code_counts(codes, len(toks))
                    nulls = int((codes < 0).sum())
                    for w, t in zip(cnt, toks):
                        if w and t:
                            np.add.at(hist, hash_terms(t, nb), w)
                else:
                    rows = P.values[k]
                    nulls = sum(1 for r in rows if r is None)
                    for r in rows:
                        if r:
                            np.add.at(hist, hash_terms(r, nb), 1.0)
                if k in P.text_codes:
                    pairs = [(x, int(w)) for w, t in zip(cnt, toks) if w for x in (t or ())]
                    card = _text_stats([x for x, _ in pairs], [w for _, w in pairs])
                else:
                    card = _text_stats(x for r in rows if r for x in r)
                dists[k] = FeatureDistribution(k[0], k[1], n, nulls, hist, [sm.min, sm.max, sm.sum, sm.count],
                                               _moments_from_sums(*power[k]), dist_type, card)
            else:
                rows = P.values[k]
                nulls = sum(1 for r in rows if r is None)
                flat = np.asarray([x for r in rows if r is not None for x in r], np.float64)
                if sm.is_empty:
                    info_v, hist = [sm.min, sm.max], np.zeros(0)
                elif sm.min < sm.max:
                    step = (sm.max - sm.min) / (self.bins - 2.0)
                    splits = np.array([sm.min + step * b for b in range(self.bins)])
                    b = np.searchsorted(splits, flat, side="right") - 1
                    b = np.where((flat >= splits[0]) & (flat < splits[-1]), b, self.bins - 1)
                    info_v, hist = splits.tolist(), np.bincount(b, minlength=self.bins).astype(np.float64)
                else:
                    info_v = [sm.min, sm.max, sm.sum, sm.count]
                    hist = np.array([float((flat == sm.max).sum()), float((flat != sm.max).sum())])
                dists[k] = FeatureDistribution(k[0], k[1], n, nulls, hist, info_v, _moments_from_sums(*power[k]),
                                               dist_type, _text_stats(flat.tolist()))
        # ---- null-indicator / label leakage correlations
        if info is not None:
            corr = info.correlation_info
        else:
            corr = {}
            for rk in resp_keys:
                y = P.response_value.get(rk)
                if y is None:
                    continue
                corr[rk] = self._null_label_corr(y, P, pred_keys, stats)
        resp_sum = OrderedDict((k, summaries[k]) for k in resp_keys)
        pred_sum = OrderedDict((k, summaries[k]) for k in pred_keys)
        if info is not None:
            resp_sum, pred_sum = info.response_summaries, info.predictor_summaries
        return AllFeatureInformation(resp_sum, [dists[k] for k in resp_keys if k in dists], pred_sum,
                                     [dists[k] for k in pred_sum if k in dists], corr)

    def _null_label_corr(self, y: torch.Tensor, P: _Prepared, pred_keys, stats) -> Dict[FeatureKey, float]:
        n = float(P.n)
        yv = y.to(torch.float64)
        if self.correlation_type == "spearman":
            yv = _avg_ranks(yv)
        sy = float(yv.sum())
        syy = float((yv * yv).sum())
        out = {}
        for k in pred_keys:
            if k in P.nulls:
                z = P.nulls[k]
                yz = yv.to(z.device)
                sz = float(z.sum())
                syz = float(yz[z].sum())
            else:
                zl = [r is None for r in P.values[k]]
                z = torch.tensor(zl, dtype=torch.bool)
                sz = float(z.sum())
                syz = float(yv.cpu()[z].sum())
            num = n * syz - sy * sz
            den = math.sqrt(max(n * syy - sy * sy, 0.0) * max(n * sz - sz * sz, 0.0))
            c = num / den if den > 0 else float("nan")
            out[k] = min(abs(c), 1.0) if not math.isnan(c) else float("nan")
        return out

    # ----------------------------------------------------------------------------------- decisions
    def metrics_and_reasons(self, train: List[FeatureDistribution], score: List[FeatureDistribution],
                            corr_info) -> Tuple[List[RawFeatureFilterMetrics], List[ExclusionReasons]]:
        metrics, reasons = [], []
        score_by = {d.feature_key: d for d in score}
        for t in train:
            fr = t.fill_rate()
            corrs = [c.get(t.feature_key) for c in corr_info.values()]
            nl = next((c for c in corrs if c is not None), None) if corrs else None
            s = score_by.get(t.feature_key) if score else None
            m = RawFeatureFilterMetrics(t.name, t.key, fr, nl, None if s is None else s.fill_rate(),
                                        None if s is None else t.js_divergence(s),
                                        None if s is None else t.relative_fill_rate(s),
                                        None if s is None else t.relative_fill_ratio(s))
            metrics.append(m)
            tu = fr < self.min_fill
            leak = nl is not None and not math.isnan(nl) and nl > self.max_correlation
            su = m.scoringFillRate is not None and m.scoringFillRate < self.min_fill
            js = (t.name not in self.js_protected and m.jsDivergence is not None
                  and m.jsDivergence > self.max_js_divergence)
            fd = m.fillRateDiff is not None and m.fillRateDiff > self.max_fill_difference
            fq = m.fillRatioDiff is not None and m.fillRatioDiff > self.max_fill_ratio_diff
            reasons.append(ExclusionReasons(t.name, t.key, tu, leak, su, js, fd, fq,
                                            any([tu, leak, su, js, fd, fq])))
        return metrics, reasons

    def features_to_exclude(self, train, score, corr_info):
        metrics, reasons = self.metrics_and_reasons(train, score, corr_info)
        drop = {}
        keep = {}
        for t, r in zip(train, reasons):
            (drop if r.excluded else keep).setdefault(t.name, []).append(t)
        map_names = set(drop) & set(keep)
        to_drop_names = [k for k in drop if k not in map_names]
        to_drop_keys = {k: {d.key for d in drop[k] if d.key is not None} for k in drop if k in map_names}
        return metrics, reasons, to_drop_names, to_drop_keys

    # -------------------------------------------------------------------------------------- driver
    def generate_filtered_raw(self, raw_features, params=None, train_ds: Optional[Dataset] = None):
        """Returns ``(cleaned dataset, features to drop, map keys to drop, results)``."""
        if train_ds is None:
            train_ds = self.training_reader.generate_dataset(raw_features, params)
        if len(train_ds) == 0:
            raise ValueError("RawFeatureFilter cannot work with empty training data")
        stats_ds = train_ds
        if getattr(train_ds, "sharded", False):
            # row-sharded input: the distributions are computed on the gathered raw columns so every
            # rank derives the identical blocklist (the filtered DAG must agree across ranks)
            from ..parallel import dp
            with dp.scope(True):
                stats_ds = dp.gather_dataset(train_ds, [n for n in train_ds.names])
        tinfo = self.compute_feature_stats(stats_ds, raw_features, TRAINING)
        sinfo = None
        if self.scoring_reader is not None:
            sds = self.scoring_reader.generate_dataset(raw_features, params)
            if len(sds) >= self.min_scoring_rows:
                sinfo = self.compute_feature_stats(sds, raw_features, SCORING, tinfo)
        tp = [d for d in tinfo.predictor_distributions if d.name not in self.protected]
        sp = [d for d in sinfo.predictor_distributions if d.name not in self.protected] if sinfo else []
        metrics, reasons, drop_names, drop_keys = self.features_to_exclude(tp, sp, tinfo.correlation_info)
        to_drop = [f for f in raw_features if f.name in drop_names]
        kept = [f for f in raw_features if f.name not in drop_names]
        if not any(not f.is_response for f in kept):
            raise ValueError("The raw feature filter has dropped all of your features, check your input data quality")
        cleaned = train_ds.drop([f.name for f in to_drop])
        if drop_keys:
            cols = dict(cleaned.columns)
            for name, keys in drop_keys.items():
                c = cols[name]
                vals = [None if v is None else {k: x for k, x in v.items() if k not in keys} for v in c.to_list()]
                cols[name] = ObjectColumn(c.ftype, vals)
            cleaned = cleaned.with_columns(cols)
        cfg = RawFeatureFilterConfig(self.min_fill, self.max_fill_difference, self.max_fill_ratio_diff,
                                     self.max_js_divergence, self.max_correlation, self.correlation_type,
                                     sorted(self.js_protected), sorted(self.protected))
        dists = (tinfo.response_distributions + tinfo.predictor_distributions +
                 ((sinfo.response_distributions + sinfo.predictor_distributions) if sinfo else []))
        results = RawFeatureFilterResults(cfg, dists, metrics, reasons)
        return cleaned, to_drop, drop_keys, results


def _raw_names(f):
    if isinstance(f, str):
        return [f]
    return [r.name for r in f.raw_features()]


def _code_counts(codes: torch.Tensor, V: int) -> np.ndarray:
    c = codes.long()
    c = c[c >= 0]
    if V == 0:
        return np.zeros(0)
    return torch.bincount(c, minlength=V).to(torch.float64).cpu().numpy()[:V]


def _avg_ranks(v: torch.Tensor) -> torch.Tensor:
    s, order = torch.sort(v, stable=True)
    _, inv, cnt = torch.unique_consecutive(s, return_inverse=True, return_counts=True)
    ends = torch.cumsum(cnt, 0).to(torch.float64)
    avg = ends - (cnt.to(torch.float64) - 1) / 2.0
    r = torch.empty_like(v, dtype=torch.float64)
    r[order] = avg[inv]
    return r
