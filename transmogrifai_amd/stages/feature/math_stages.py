"""Numeric transformers: arithmetic, unary math, scaling, filling, bucketizing, calibration.

Reference: ``MathTransformers.scala:50-393`` (plus / minus / multiply / divide, scalar variants, abs, ceil,
floor, round, exp, sqrt, log, power, roundDigits), ``FillMissingWithMean.scala:47``,
``OpScalarStandardScaler.scala:49``, ``ScalerTransformer.scala:144`` / ``DescalerTransformer.scala:56-92``,
``PercentileCalibrator.scala:48``, ``NumericBucketizer.scala:54-300`` (binary search over splits,
one-hot + invalid + null slots) and ``IsotonicRegressionCalibrator.scala:44-63``. All ops are
whole-column tensor expressions (validity masks carried alongside values).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch

from ...config import vector_dtype
from ...data.columns import NumericColumn, VectorColumn
from ...data.vector_metadata import NULL_STRING, OTHER_STRING, OpVectorColumnMetadata, OpVectorMetadata
from ...features import types as T
from ..base import (BinaryEstimator, BinaryTransformer, OpTransformer, UnaryEstimator, UnaryTransformer,
                    register_stage)


def _f64(c: NumericColumn):
    return c.values.to(torch.float64), c.valid


def _finite(v):
    return ~(torch.isnan(v) | torch.isinf(v))


@register_stage
class BinaryMathTransformer(BinaryTransformer):
    """plus / minus / multiply / divide of two numeric columns -> Real."""
    output_type = T.Real
    _defaults = {"op": "plus"}

    def __init__(self, op: str = "plus", uid=None, **kw):
        super().__init__(None, uid=uid, operation_name=op, op=op, **kw)

    def transform_columns(self, a, b, ds=None):
        x, xa = _f64(a)
        y, ya = _f64(b)
        op = self.params["op"]
        if op == "plus":
            v = torch.where(xa & ya, x + y, torch.where(xa, x, y))
            ok = xa | ya
        elif op == "minus":
            v = torch.where(xa & ya, x - y, torch.where(xa, x, -y))
            ok = xa | ya
        elif op == "multiply":
            v = x * y
            ok = xa & ya & _finite(v)
        elif op == "divide":
            v = x / y
            ok = xa & ya & _finite(v)
        else:
            raise ValueError(op)
        return NumericColumn(T.Real, torch.where(ok, v, torch.zeros_like(v)), ok)

    def transform_row(self, a, b):
        col = self.transform_columns(NumericColumn.from_values(T.Real, [a]), NumericColumn.from_values(T.Real, [b]))
        return col.row(0)


@register_stage
class ScalarMathTransformer(UnaryTransformer):
    """``x op scalar`` (or ``scalar op x`` when reversed) -> Real."""
    output_type = T.Real
    _defaults = {"op": "plus", "scalar": 0.0, "reverse": False}

    def __init__(self, op: str = "plus", scalar: float = 0.0, reverse: bool = False, uid=None, **kw):
        super().__init__(None, uid=uid, operation_name=op + "S", op=op, scalar=float(scalar), reverse=reverse, **kw)

    def transform_columns(self, a, ds=None):
        x, ok = _f64(a)
        s = self.params["scalar"]
        op = self.params["op"]
        rev = self.params["reverse"]
        if op == "plus":
            v = x + s
        elif op == "minus":
            v = (s - x) if rev else (x - s)
        elif op == "multiply":
            v = x * s
        elif op == "divide":
            v = (s / x) if rev else (x / s)
        elif op == "power":
            v = torch.pow(torch.full_like(x, s), x) if rev else torch.pow(x, s)
        else:
            raise ValueError(op)
        ok = ok & _finite(v)
        return NumericColumn(T.Real, torch.where(ok, v, torch.zeros_like(v)), ok)

    def transform_row(self, a):
        return self.transform_columns(NumericColumn.from_values(T.Real, [a])).row(0)


def java_round(x: torch.Tensor) -> torch.Tensor:
    """``math.round`` (Java ``Math.round``): the nearest integer, halves toward +inf (2.5 -> 3, -2.5 -> -2) --
    not torch's half-to-even. Written as floor + a compare of the exact fraction ``x - floor(x)``, so
    0.49999999999999994 rounds to 0 as in Java (``floor(x + 0.5)`` would give 1)."""
    f = torch.floor(x)
    return torch.where(x - f >= 0.5, f + 1, f)


_UNARY = {"abs": torch.abs, "ceil": torch.ceil, "floor": torch.floor, "round": java_round, "exp": torch.exp,
          "sqrt": torch.sqrt, "log": None, "sigmoid": torch.sigmoid}


@register_stage
class UnaryMathTransformer(UnaryTransformer):
    output_type = T.Real
    _defaults = {"op": "abs", "base": math.e, "digits": 0}

    def __init__(self, op: str = "abs", uid=None, **kw):
        super().__init__(None, uid=uid, operation_name=op, op=op, **kw)
        if op in ("ceil", "floor", "round"):
            self.output_type = T.Integral
        if op == "log" and not self.params["base"] > 0:
            raise ValueError("requirement failed: log base must be greater than 0")

    def transform_columns(self, a, ds=None):
        x, ok = _f64(a)
        op = self.params["op"]
        if op == "log":       # LogTransformer (MathTransformers.scala:343): log10(v) / log10(base)
            v = torch.log10(x) / math.log10(self.params["base"])
        elif op == "roundDigits":   # RoundDigitsTransformer (:388): math.round(v * 10^d) / 10^d
            f = math.pow(10.0, self.params["digits"])
            v = java_round(x * f) / f
        else:
            v = _UNARY[op](x)
        ok = ok & _finite(v)
        if op in ("ceil", "floor", "round"):
            return NumericColumn(T.Integral, torch.where(ok, v, torch.zeros_like(v)).to(torch.int64), ok)
        return NumericColumn(T.Real, torch.where(ok, v, torch.zeros_like(v)), ok)

    def transform_row(self, a):
        return self.transform_columns(NumericColumn.from_values(T.Real, [a])).row(0)


# ---------------------------------------------------------------------------------------- fills
@register_stage
class FillMissingWithMeanModel(UnaryTransformer):
    operation_name = "fillWithMean"
    output_type = T.RealNN

    def __init__(self, mean: float = 0.0, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.mean = mean

    def transform_columns(self, a, ds=None):
        x, ok = _f64(a)
        return NumericColumn(T.RealNN, torch.where(ok, x, torch.full_like(x, self.mean)),
                             torch.ones_like(ok))

    def transform_row(self, a):
        return float(a) if a is not None else self.mean

    def ctor_args(self):
        return {"mean": self.mean}

    def load_ctor_args(self, a):
        self.mean = a["mean"]


@register_stage
class FillMissingWithMean(UnaryEstimator):
    operation_name = "fillWithMean"
    output_type = T.RealNN
    _defaults = {"default_value": 0.0}

    def fit_columns(self, a, ds=None):
        x, ok = _f64(a)
        n = int(ok.sum())
        m = float(x[ok].mean()) if n > 0 else float(self.params["default_value"])
        return FillMissingWithMeanModel(m)


@register_stage
class OpScalarStandardScalerModel(UnaryTransformer):
    operation_name = "stdScaled"
    output_type = T.RealNN

    def __init__(self, mean: float = 0.0, std: float = 1.0, with_mean=True, with_std=True, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.mean, self.std, self.with_mean, self.with_std = mean, std, with_mean, with_std

    def transform_columns(self, a, ds=None):
        x, ok = _f64(a)
        v = x - self.mean if self.with_mean else x
        if self.with_std:
            v = v / self.std if self.std != 0 else torch.zeros_like(v)
        return NumericColumn(T.RealNN, torch.where(ok, v, torch.zeros_like(v)), torch.ones_like(ok))

    def transform_row(self, a):
        return self.transform_columns(NumericColumn.from_values(T.Real, [a])).row(0)

    def ctor_args(self):
        return {"mean": self.mean, "std": self.std, "withMean": self.with_mean, "withStd": self.with_std}

    def load_ctor_args(self, a):
        self.mean, self.std, self.with_mean, self.with_std = a["mean"], a["std"], a["withMean"], a["withStd"]


@register_stage
class OpScalarStandardScaler(UnaryEstimator):
    """z-normalization (``RichNumericFeature.zNormalize``)."""
    operation_name = "stdScaled"
    output_type = T.RealNN
    _defaults = {"with_mean": True, "with_std": True}

    def fit_columns(self, a, ds=None):
        x, ok = _f64(a)
        v = x[ok]
        mean = float(v.mean()) if v.numel() else 0.0
        std = float(v.std(unbiased=True)) if v.numel() > 1 else 0.0
        # the descaler's view of the fit (OpScalarStandardScaler.scala fitFn): linear, 1 / std, -mean / std
        slope = 1.0 / std if std != 0 else float("inf")
        self.metadata.update(scaler_metadata("Linear", slope, -mean * slope if std != 0 else float("-inf")))
        return OpScalarStandardScalerModel(mean, std, self.params["with_mean"], self.params["with_std"])


SCALING_TYPE_KEY, SCALING_ARGS_KEY = "scalingType", "scalingArgs"


def scaler_metadata(scaling_type: str, slope: float = 1.0, intercept: float = 0.0) -> dict:
    """``ScalerMetadata.toMetadata`` (ScalerTransformer.scala): the scaling family and its JSON arguments."""
    import json
    args = {"slope": float(slope), "intercept": float(intercept)} if scaling_type == "Linear" else {}
    return {SCALING_TYPE_KEY: scaling_type, SCALING_ARGS_KEY: json.dumps(args, separators=(",", ":"))}


def parse_scaler_metadata(meta: dict) -> Optional[dict]:
    """(scaling_type, slope, intercept) params from stage metadata written by ``scaler_metadata``, or None."""
    import json
    if not meta or SCALING_TYPE_KEY not in meta:
        return None
    args = json.loads(meta.get(SCALING_ARGS_KEY) or "{}")
    return {"scaling_type": meta[SCALING_TYPE_KEY], "slope": float(args.get("slope", 1.0)),
            "intercept": float(args.get("intercept", 0.0))}


def _check_linear(p):
    if p.get("scaling_type", "Linear") == "Linear" and float(p.get("slope", 1.0)) == 0.0:
        raise ValueError("requirement failed: LinearScaler must have a non-zero slope to be invertible")


@register_stage
class ScalerTransformer(UnaryTransformer):
    """Linear (``slope * x + intercept``) or log scaling with stored args (``ScalerTransformer.scala``)."""
    operation_name = "scaler"
    output_type = T.Real
    _defaults = {"scaling_type": "Linear", "slope": 1.0, "intercept": 0.0}

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        _check_linear(self.params)
        self.metadata.update(scaler_metadata(self.params["scaling_type"], self.params["slope"],
                                             self.params["intercept"]))

    def set(self, name, value):
        super().set(name, value)
        if name in ("scaling_type", "slope", "intercept"):
            _check_linear(self.params)
        if name in ("scaling_type", "slope", "intercept") and "metadata" in self.__dict__:
            self.metadata.update(scaler_metadata(self.params["scaling_type"], self.params["slope"],
                                                 self.params["intercept"]))
        return self

    def transform_columns(self, a, ds=None):
        x, ok = _f64(a)
        self.metadata.update(scaler_metadata(self.params["scaling_type"], self.params["slope"],
                                             self.params["intercept"]))
        if self.params["scaling_type"] == "Logarithmic":
            v = torch.log(x)
        else:
            v = self.params["slope"] * x + self.params["intercept"]
        ok = ok & _finite(v)
        return NumericColumn(T.Real, torch.where(ok, v, torch.zeros_like(v)), ok)

    def transform_row(self, a):
        return self.transform_columns(NumericColumn.from_values(T.Real, [a])).row(0)


@register_stage
class DescalerTransformer(BinaryTransformer):
    """Inverse of the scaling recorded in the metadata of the second input (``DescalerTransformer.scala``): the
    ``ScalerMetadata`` of its origin stage -- a ``ScalerTransformer``, or a fitted ``OpScalarStandardScaler``
    (linear, slope 1 / std, intercept -mean / std). The resolved scaling is kept in this stage's params, so a
    saved model descales without its input's stage."""
    operation_name = "descaler"
    output_type = T.Real
    _defaults = {"scaling_type": "Linear", "slope": 1.0, "intercept": 0.0}

    def _resolve_scaling(self):
        if len(self._inputs) > 1:
            st = self._inputs[1].origin_stage
            sc = parse_scaler_metadata(getattr(st, "metadata", None) or {})
            if sc is not None:
                self.params.update(sc)

    def transform_columns(self, a, b=None, ds=None):
        x, ok = _f64(a)
        self._resolve_scaling()
        if self.params["scaling_type"] == "Logarithmic":
            v = torch.exp(x)
        else:
            v = (x - self.params["intercept"]) / self.params["slope"]
        ok = ok & _finite(v)
        return NumericColumn(T.Real, torch.where(ok, v, torch.zeros_like(v)), ok)


@register_stage
class PredictionDescaler(DescalerTransformer):
    """Descale a model's ``Prediction`` back to the original label scale with the scaling of the second
    input's ``ScalerTransformer`` (``DescalerTransformer.scala:92-112``): the prediction value of the
    Prediction map goes through the inverse scaling; raw / probability are dropped."""
    operation_name = "descaler"
    output_type = T.Real

    def transform_columns(self, a, b=None, ds=None):
        from ...data.columns import PredictionColumn
        if isinstance(a, PredictionColumn):
            p = a.prediction.to(torch.float64)
            a = NumericColumn(T.Real, p, torch.ones(p.shape[0], dtype=torch.bool, device=p.device))
        return super().transform_columns(a, b, ds=ds)

    def transform_row(self, *values):
        v = values[0]
        if isinstance(v, dict):
            v = v.get("prediction")
        elif isinstance(v, T.FeatureType):
            v = v.value.get("prediction") if isinstance(v.value, dict) else v.value
        return self.transform_columns(NumericColumn.from_values(T.Real, [v])).row(0)


# ------------------------------------------------------------------------------------ bucketizer
def java_double(v: float) -> str:
    """Java ``Double.toString`` formatting (bucket labels must match the reference)."""
    v = float(v)
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    if math.isnan(v):
        return "NaN"
    if v == 0:
        return "0.0" if math.copysign(1, v) > 0 else "-0.0"
    if 1e-3 <= abs(v) < 1e7:
        return repr(v)
    m, e = np.format_float_scientific(v, unique=True, trim="-").split("e")
    if "." not in m:
        m += ".0"
    return f"{m}E{int(e)}"


def bucket_labels(splits: Sequence[float], inclusion: str = "Left") -> List[str]:
    pre, suf = ("[", ")") if inclusion == "Left" else ("(", "]")
    return [f"{pre}{java_double(a)}-{java_double(b)}{suf}" for a, b in zip(splits[:-1], splits[1:])]


def check_splits(splits: Sequence[float]) -> bool:
    if len(splits) < 3:
        return False
    return all(a < b and not math.isnan(a) for a, b in zip(splits[:-1], splits[1:]))


def bucketize_column(x: torch.Tensor, ok: torch.Tensor, splits: Sequence[float], track_nulls: bool,
                     track_invalid: bool, inclusion: str, dtype) -> torch.Tensor:
    """One-hot bucket index via binary search (``NumericBucketizer.bucketize:219-265``); HIP
    ``bucketize_kernel`` on device (``ops/text.py``)."""
    from ...ops.text import bucketize_into
    nb = len(splits) - 1
    width = nb + (1 if track_invalid else 0) + (1 if track_nulls else 0)
    out = torch.zeros(x.shape[0], width, dtype=dtype, device=x.device)
    bucketize_into(out, x, ok, splits, track_nulls, track_invalid, inclusion == "Left")
    return out


def bucket_metadata(tf, labels, track_nulls, track_invalid) -> List[OpVectorColumnMetadata]:
    base = dict(parent_feature_name=(tf.name,), parent_feature_type=(tf.type_name,), grouping=tf.name)
    cols = [OpVectorColumnMetadata(indicator_value=l, **base) for l in labels]
    if track_invalid:
        cols.append(OpVectorColumnMetadata(indicator_value=OTHER_STRING, **base))
    if track_nulls:
        cols.append(OpVectorColumnMetadata(indicator_value=NULL_STRING, **base))
    return cols


@register_stage
class NumericBucketizer(OpTransformer):
    operation_name = "numBuck"
    output_type = T.OPVector
    arity = 1
    _defaults = {"splits": [float("-inf"), 0.0, float("inf")], "bucket_labels": None, "track_nulls": True,
                 "track_invalid": False, "split_inclusion": "Left"}

    # NumericBucketizerParams (NumericBucketizer.scala): splits validated by checkSplits (>= 3 points, strictly
    # increasing, no NaN), labels one fewer than the splits; labels derived from the splits follow a later
    # change of the split inclusion, explicit ones stay
    def set(self, name, value):
        if name == "splits" and value is not None and not check_splits([float(v) for v in value]):
            raise ValueError(f"invalid splits {list(value)}: need >= 3 strictly increasing points, no NaN")
        if name == "split_inclusion" and value not in ("Left", "Right"):
            raise ValueError(f"split_inclusion must be 'Left' or 'Right', got {value!r}")
        return super().set(name, value)

    def set_buckets(self, splits, bucket_labels=None) -> "NumericBucketizer":
        splits = [float(v) for v in splits]
        if not check_splits(splits):
            raise ValueError(f"invalid splits {splits}: need >= 3 strictly increasing points, no NaN")
        if bucket_labels is not None and len(bucket_labels) != len(splits) - 1:
            raise ValueError("The number of labels should be one less than the number of split points")
        self.set("splits", splits)
        return self.set("bucket_labels", list(bucket_labels) if bucket_labels is not None else None)

    def get_splits(self) -> List[float]:
        return [float(v) for v in self.params["splits"]]

    def get_bucket_labels(self) -> List[str]:
        return list(self.params["bucket_labels"] or bucket_labels(self.get_splits(), self.params["split_inclusion"]))

    def transform_columns(self, a, ds=None):
        p = self.params
        splits = [float(v) for v in p["splits"]]
        x, ok = _f64(a)
        labels = p["bucket_labels"] or bucket_labels(splits, p["split_inclusion"])
        if len(labels) != len(splits) - 1:
            raise ValueError("The number of labels should be one less than the number of split points")
        if self._inputs:
            t = self.get_transient_features()[0]
            self.metadata["vector_metadata"] = OpVectorMetadata(
                self.get_output_feature_name(), bucket_metadata(t, labels, p["track_nulls"], p["track_invalid"]),
                {t.name: __import__("transmogrifai_amd.data.vector_metadata", fromlist=["FeatureHistory"])
                 .FeatureHistory(tuple(t.origin_features), tuple(t.stages) + (self.stage_name(),))})
        out = bucketize_column(x, ok, splits, p["track_nulls"], p["track_invalid"], p["split_inclusion"],
                               vector_dtype(x.device))
        return VectorColumn(out, self.metadata.get("vector_metadata"))


@register_stage
class PercentileCalibratorModel(UnaryTransformer):
    """Percentile bucket of a score (``PercentileCalibrator.scala`` ``PercentileCalibratorModel``): the insertion
    index of the score in the quantile splits, rescaled to 0 .. expectedNumBuckets - 1 when fewer distinct
    splits than expected buckets were found."""
    operation_name = "percentCalibrator"
    output_type = T.RealNN

    def __init__(self, splits=None, actual_num_buckets=None, expected_num_buckets=100, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.splits = [float(v) for v in (splits or [])]
        self.actual_num_buckets = len(self.splits) if actual_num_buckets is None else int(actual_num_buckets)
        self.expected_num_buckets = int(expected_num_buckets)

    def calibrate(self, x: torch.Tensor) -> torch.Tensor:
        s = torch.as_tensor(self.splits, dtype=torch.float64, device=x.device)
        idx = torch.searchsorted(s, x.to(torch.float64), right=False).to(torch.float64)   # Found / InsertionPoint
        act, exp = self.actual_num_buckets, self.expected_num_buckets
        if act >= exp:
            return idx - 1.0                                            # start at zero
        old_max, new_max = max(act - 2, 0), max(exp - 1, 0)
        if old_max == 0:
            return torch.zeros_like(idx)
        v = torch.floor(idx * float(new_max) / old_max + 0.5)            # Scala Double.round
        return torch.clamp(v, max=float(new_max))

    def transform_columns(self, a, ds=None):
        x, ok = _f64(a)
        v = self.calibrate(x)
        return NumericColumn(T.RealNN, torch.where(ok, v, torch.zeros_like(v)), torch.ones_like(ok))

    def ctor_args(self):
        return {"splits": self.splits, "actualNumBuckets": self.actual_num_buckets,
                "expectedNumBuckets": self.expected_num_buckets}

    def load_ctor_args(self, a):
        self.splits = [float(v) for v in a["splits"]]
        self.actual_num_buckets = int(a.get("actualNumBuckets", len(self.splits)))
        self.expected_num_buckets = int(a.get("expectedNumBuckets", 100))


ORIG_SPLITS_KEY, SCALED_SPLITS_KEY = "origSplits", "scaledSplits"


def exact_quantile_splits(v: torch.Tensor, num_buckets: int) -> List[float]:
    """Spark ``QuantileDiscretizer`` with relativeError 0: the exact quantiles at 0, 1/k, .., 1 (the element of
    rank ceil(p n)), ends replaced by -Inf / +Inf, duplicates dropped."""
    vs = torch.sort(v.to(torch.float64)).values
    n = vs.numel()
    step = 1.0 / num_buckets
    ps = [0.0 + step * i for i in range(num_buckets + 1)]
    idx = [0 if p <= 0 else n - 1 if p >= 1 else min(max(math.ceil(p * n) - 1, 0), n - 1) for p in ps]
    q = vs[torch.as_tensor(idx, device=vs.device)].tolist()
    q[0], q[-1] = float("-inf"), float("inf")
    return sorted(set(q))


@register_stage
class PercentileCalibrator(UnaryEstimator):
    """Map a score to its percentile bucket (``PercentileCalibrator.scala``): exact quantile splits of the
    scores, the calibrated split values recorded in the summary metadata (origSplits / scaledSplits)."""
    operation_name = "percentCalibrator"
    output_type = T.RealNN
    _defaults = {"expected_num_buckets": 100}

    def fit_columns(self, a, ds=None):
        x, ok = _f64(a)
        v = x[ok]
        k = int(self.params["expected_num_buckets"])
        splits = exact_quantile_splits(v, k) if v.numel() else [float("-inf"), float("inf")]
        model = PercentileCalibratorModel(splits, len(splits), k)
        scaled = model.calibrate(torch.as_tensor(splits, dtype=torch.float64)).tolist()
        self.metadata["summary"] = {ORIG_SPLITS_KEY: [java_double(s) for s in splits],
                                    SCALED_SPLITS_KEY: [java_double(s) for s in scaled]}
        return model


@register_stage
class IsotonicRegressionCalibratorModel(BinaryTransformer):
    operation_name = "isotonic"
    output_type = T.RealNN
    allow_label_as_input = True

    def __init__(self, boundaries=None, predictions=None, uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.boundaries = list(boundaries or [])
        self.predictions = list(predictions or [])

    def transform_columns(self, label, a, ds=None):
        x, ok = _f64(a)
        bx = torch.as_tensor(self.boundaries, dtype=torch.float64, device=x.device)
        by = torch.as_tensor(self.predictions, dtype=torch.float64, device=x.device)
        v = _interp(x, bx, by)
        return NumericColumn(T.RealNN, torch.where(ok, v, torch.zeros_like(v)), torch.ones_like(ok))

    def ctor_args(self):
        return {"boundaries": self.boundaries, "predictions": self.predictions}

    def load_ctor_args(self, a):
        self.boundaries, self.predictions = list(a["boundaries"]), list(a["predictions"])


def _interp(x, bx, by):
    if bx.numel() == 0:
        return torch.zeros_like(x)
    if bx.numel() == 1:
        return torch.full_like(x, float(by[0]))
    i = torch.searchsorted(bx, x).clamp(1, bx.numel() - 1)
    x0, x1, y0, y1 = bx[i - 1], bx[i], by[i - 1], by[i]
    t = torch.where(x1 > x0, (x - x0) / (x1 - x0), torch.zeros_like(x))
    v = y0 + t * (y1 - y0)
    v = torch.where(x <= bx[0], by[0], v)
    return torch.where(x >= bx[-1], by[-1], v)


def pava(x: np.ndarray, y: np.ndarray, w: Optional[np.ndarray] = None, increasing: bool = True):
    """Pool-adjacent-violators isotonic fit; returns (boundaries, predictions) like Spark."""
    order = np.lexsort((y, x))
    x, y = x[order], y[order]
    w = np.ones_like(y) if w is None else w[order]
    if not increasing:
        y = -y
    vals, wts, lo, hi = [], [], [], []
    for i in range(len(x)):
        vals.append(y[i]); wts.append(w[i]); lo.append(x[i]); hi.append(x[i])
        while len(vals) > 1 and vals[-2] > vals[-1]:
            v = (vals[-2] * wts[-2] + vals[-1] * wts[-1]) / (wts[-2] + wts[-1])
            wt = wts[-2] + wts[-1]
            h1 = hi[-1]
            vals.pop(); wts.pop(); lo.pop(); hi.pop()
            vals[-1], wts[-1], hi[-1] = v, wt, h1        # the pooled block spans [lo of the first, hi of the last]
    # Spark's compression: adjacent points with the same prediction keep only their two boundary points
    runs = []
    for v, l, h in zip(vals, lo, hi):
        if runs and runs[-1][0] == v:
            runs[-1][2] = h
        else:
            runs.append([v, l, h])
    bnd, pred = [], []
    for v, l, h in runs:
        vv = v if increasing else -v
        bnd.append(l); pred.append(vv)
        if h > l:
            bnd.append(h); pred.append(vv)
    return bnd, pred


@register_stage
class IsotonicRegressionCalibrator(BinaryEstimator):
    operation_name = "isotonic"
    output_type = T.RealNN
    allow_label_as_input = True
    _defaults = {"isotonic": True}

    def fit_columns(self, label, a, ds=None):
        x, ok = _f64(a)
        y = label.values.to(torch.float64)
        b, p = pava(x[ok].cpu().numpy(), y[ok].cpu().numpy(), increasing=self.params["isotonic"])
        return IsotonicRegressionCalibratorModel(b, p)
