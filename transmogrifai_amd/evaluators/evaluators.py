"""Evaluators and the ``Evaluators`` factory.

Reference: ``core/.../evaluators/Evaluators.scala:51-319`` (factory), ``OpBinaryClassificationEvaluator``
(``:56-174``), ``OpBinScoreEvaluator`` (``:60-173``), ``OpMultiClassificationEvaluator``,
``OpRegressionEvaluator``, ``OpForecastEvaluator`` and ``OPLogLoss``. An evaluator reads the label
and ``Prediction`` columns of a dataset (or raw arrays, which is how the model selector calls it)
and returns a metrics dict; ``evaluate`` returns the single selection metric.
"""
from __future__ import annotations

import os

from typing import Callable, Dict, Optional

import torch

from ..data.columns import PredictionColumn
from . import metrics as M


class OpEvaluatorBase:
    name = "evaluator"
    default_metric = ""
    larger_better = True

    def __init__(self, metric: Optional[str] = None, uid: Optional[str] = None, **kw):
        from ..uid import make_uid
        self.uid = uid or make_uid(type(self).__name__)
        self.metric = metric or self.default_metric
        self.label_col = None
        self.prediction_col = None
        self.params = kw

    def set_label_col(self, f):
        self.label_col = f.name if hasattr(f, "name") else f
        return self

    def set_prediction_col(self, f):
        self.prediction_col = f.name if hasattr(f, "name") else f
        return self

    @property
    def is_larger_better(self) -> bool:
        return self.larger_better

    def _arrays(self, ds):
        y = ds[self.label_col].values.to(torch.float64)
        p: PredictionColumn = ds[self.prediction_col]
        return y, p.prediction, p.raw, p.probability

    def evaluate_all(self, ds) -> Dict:
        return self.evaluate_arrays(*self._arrays(ds))

    def evaluate(self, ds) -> float:
        return self.metric_value(self.evaluate_all(ds))

    def metric_value(self, metrics: Dict) -> float:
        return float(metrics[self.metric])

    def evaluate_arrays(self, y, pred, raw, prob) -> Dict:
        raise NotImplementedError

    def selection_metric(self, y, pred, raw, prob) -> float:
        """Metric used by the model selector on a validation fold."""
        return self.metric_value(self.evaluate_arrays(y, pred, raw, prob))

    def to_json(self):
        return {"className": type(self).__name__, "uid": self.uid, "metric": self.metric, "name": self.name}


def _score(raw, prob, pred):
    if prob is not None and prob.numel() and prob.shape[1] >= 2:
        return prob[:, 1]
    if raw is not None and raw.numel() and raw.shape[1] >= 2:
        return raw[:, 1]
    return pred


class OpBinaryClassificationEvaluator(OpEvaluatorBase):
    name = "binEval"
    default_metric = "AuROC"

    def __init__(self, metric=None, num_bins: int = 100, **kw):
        super().__init__(metric, **kw)
        self.num_bins = num_bins
        self.larger_better = self.metric not in ("Error",)

    def evaluate_arrays(self, y, pred, raw, prob):
        return M.binary_classification_metrics(pred, _score(None, prob, pred), y, self.num_bins)

    def selection_metric_batch(self, y, outputs):
        """Selection metric of several models scored on the same validation rows (``outputs`` = their
        ``(pred, raw, prob)``): AuPR / AuROC from one segmented sort of all score sets
        (:func:`metrics.binary_areas_batch`); ``None`` for the other metrics."""
        if self.metric not in ("AuPR", "AuROC") or not outputs:
            return None
        sc = [(raw[:, 1] if (raw is not None and raw.numel() and raw.shape[1] >= 2)
               else _score(raw, prob, pred)).reshape(-1) for pred, raw, prob in outputs]
        # fp32 scores stay fp32 (one packed-key sort); anything else is compared in fp64
        S = torch.stack(sc) if all(t.dtype == torch.float32 for t in sc) else \
            torch.stack([t.to(torch.float64) for t in sc])
        if S.is_cuda:       # one HIP launch for all curves (metric_kernels.hip)
            aupr, auroc = M.binary_areas_device(S, y)
        elif os.environ.get("TMOG_BATCH_METRIC") == "1":
            aupr, auroc = M.binary_areas_batch(S, y)
        else:               # host: one curve per model (binary_curves)
            return [M.binary_curves(t, y, 0)[self.metric] for t in sc]
        return (aupr if self.metric == "AuPR" else auroc).tolist()

    @property
    def batch_default(self) -> bool:
        """The validator scores all models of a fold in one batch by default on the GPU (the HIP curve kernel
        has no [J, n] torch temporaries); TMOG_BATCH_METRIC=0 / 1 overrides."""
        return self.metric in ("AuPR", "AuROC")

    def selection_metric(self, y, pred, raw, prob):
        # BinaryClassificationEvaluator on rawPrediction, exact curve (numBins = 0)
        if self.metric in ("AuPR", "AuROC"):
            s = raw[:, 1] if (raw is not None and raw.numel() and raw.shape[1] >= 2) else _score(raw, prob, pred)
            if s.is_cuda:
                return self.selection_metric_batch(y, [(pred, raw, prob)])[0]
            c = M.binary_curves(s, y, 0)
            return c[self.metric]
        if self.metric == "Error":
            tp, tn, fp, fn = M.confusion_at(pred, y)
            return (fp + fn) / max(1.0, tp + tn + fp + fn)
        return self.metric_value(self.evaluate_arrays(y, pred, raw, prob))


class OpBinScoreEvaluator(OpEvaluatorBase):
    name = "binScoreEval"
    default_metric = "BrierScore"
    larger_better = False

    def __init__(self, metric=None, num_bins: int = 100, **kw):
        super().__init__(metric, **kw)
        if not num_bins > 0:            # OpBinScoreEvaluator.scala:60
            raise ValueError("requirement failed: numOfBins must be positive")
        self.num_bins = num_bins

    def evaluate_arrays(self, y, pred, raw, prob):
        # the class-1 probability, or the class-1 raw score of a model without probabilities
        return M.bin_score_metrics(_score(raw, prob, pred), y, self.num_bins)


class OpMultiClassificationEvaluator(OpEvaluatorBase):
    name = "multiEval"
    default_metric = "F1"

    def __init__(self, metric=None, top_ns=(1, 3), thresholds=None, **kw):
        super().__init__(metric, **kw)
        self.larger_better = self.metric not in ("Error",)
        self.top_ns = list(top_ns)
        self.thresholds = None if thresholds is None else list(thresholds)

    def set_top_ns(self, top_ns):
        """``setTopNs`` (OpMultiClassificationEvaluator.scala): the top-N cut-offs of the threshold metrics."""
        self.top_ns = list(top_ns)
        return self

    def set_thresholds(self, thresholds):
        """``setThresholds``: the probability thresholds of the threshold metrics (default 0.00 .. 1.00)."""
        self.thresholds = list(thresholds)
        return self

    def evaluate_arrays(self, y, pred, raw, prob):
        return M.multiclass_metrics(pred, y, prob, top_ns=tuple(self.top_ns), thresholds=self.thresholds)

    # the selector scores every model of a fold through selection_metric_batch: the selection metric alone (the
    # full evaluation adds threshold curves over the class probabilities, ~10 ms a model on 300K-row folds)
    batch_default = True

    def selection_metric(self, y, pred, raw, prob):
        v = self.selection_metric_batch(y, [(pred, raw, prob)])
        return v[0] if v is not None else self.metric_value(self.evaluate_arrays(y, pred, raw, prob))

    def selection_metric_batch(self, y, outputs):
        """Weighted precision / recall / F1 or error of several models on the same rows from one bincount of
        (model, label, prediction) -- the arithmetic of :func:`metrics.multiclass_metrics` per model."""
        if self.metric not in ("Precision", "Recall", "F1", "Error") or not outputs:
            return None
        yi = y.to(torch.int64).reshape(-1)
        n = yi.numel()
        if n == 0:
            return [0.0] * len(outputs)
        Pm = torch.stack([p.to(device=yi.device, dtype=torch.int64).reshape(-1) for p, _, _ in outputs])   # [J, n]
        J = Pm.shape[0]
        K = int(max(int(Pm.max()), int(yi.max()))) + 1
        idx = (torch.arange(J, device=yi.device)[:, None] * K + yi[None, :]) * K + Pm
        cm = torch.bincount(idx.reshape(-1), minlength=J * K * K).view(J, K, K).to(torch.float64)
        tp = torch.diagonal(cm, dim1=1, dim2=2)
        actual, predicted = cm.sum(2), cm.sum(1)
        prec_c = torch.where(predicted > 0, tp / predicted.clamp_min(1), torch.zeros_like(tp))
        rec_c = torch.where(actual > 0, tp / actual.clamp_min(1), torch.zeros_like(tp))
        wts = actual / n
        out = []
        for prec, rec, t in zip((prec_c * wts).sum(1).tolist(), (rec_c * wts).sum(1).tolist(), tp.sum(1).tolist()):
            if self.metric == "Precision":
                out.append(prec)
            elif self.metric == "Recall":
                out.append(rec)
            elif self.metric == "F1":
                out.append(0.0 if prec + rec == 0 else 2 * prec * rec / (prec + rec))
            else:
                out.append(1.0 - t / n)
        return out


class OpRegressionEvaluator(OpEvaluatorBase):
    name = "regEval"
    default_metric = "RootMeanSquaredError"
    larger_better = False

    def __init__(self, metric=None, **kw):
        super().__init__(metric, **kw)
        self.larger_better = self.metric == "R2"
        self.bins = list(M.DEFAULT_PCT_ERROR_BINS)
        self.scaled_error_cutoff = 1e-3
        self.smart_cutoff_ratio = None

    def set_percentage_error_histogram_bins(self, bins):
        """``setPercentageErrorHistogramBins`` (OpRegressionEvaluator.scala:63-73): non-empty and sorted."""
        b = [float(x) for x in bins]
        if not b or b != sorted(b):
            raise ValueError("signedPercentageErrorHistogramBins must be non-empty and sorted")
        self.bins = b
        return self

    def set_scaled_error_cutoff(self, v: float):
        if not v >= 0.0:
            raise ValueError("scaledErrorCutoff must be non-negative")
        self.scaled_error_cutoff = float(v)
        return self

    def set_smart_cutoff_ratio(self, v: float):
        if not v >= 0.0:
            raise ValueError("smartCutoffRatio must be non-negative")
        self.smart_cutoff_ratio = float(v)
        return self

    def evaluate_arrays(self, y, pred, raw, prob):
        if self.smart_cutoff_ratio is not None:      # calculateSmartCutoff (:170-174), remembered as the reference
            yv = y.to(torch.float64).reshape(-1)
            mean_abs = float(yv.abs().mean()) if yv.numel() else 0.0
            self.scaled_error_cutoff = max(self.smart_cutoff_ratio * mean_abs, self.scaled_error_cutoff)
        return M.regression_metrics(pred, y, bins=self.bins, scaled_error_cutoff=self.scaled_error_cutoff)

    # the selector scores every model of a fold with this (no percentage-error histogram, one host read
    # for all of them): the full metric set cost ~9 ms per model on 30M-row folds, mostly device syncs
    batch_default = True

    def selection_metric(self, y, pred, raw, prob):
        v = self.selection_metric_batch(y, [(pred, raw, prob)])
        return v[0] if v is not None else self.metric_value(self.evaluate_arrays(y, pred, raw, prob))

    def selection_metric_batch(self, y, outputs):
        if self.metric not in ("RootMeanSquaredError", "MeanSquaredError", "MeanAbsoluteError", "R2") or not outputs:
            return None
        yd = y.to(torch.float64).reshape(-1)
        n = yd.numel()
        if n == 0:
            return [0.0] * len(outputs)
        ss_tot = ((yd - yd.mean()) ** 2).sum() if self.metric == "R2" else None
        vals = []
        for pred, _, _ in outputs:
            e = pred.to(torch.float64).reshape(-1) - yd
            if self.metric == "MeanAbsoluteError":
                vals.append(e.abs().mean())
                continue
            sse = (e * e).sum()
            if self.metric == "R2":
                vals.append(torch.where(ss_tot > 0, 1.0 - sse / ss_tot.clamp_min(1e-300), torch.zeros_like(sse)))
            elif self.metric == "MeanSquaredError":
                vals.append(sse / n)
            else:
                vals.append(torch.sqrt(sse / n))
        return torch.stack(vals).tolist()


class OpForecastEvaluator(OpEvaluatorBase):
    name = "forecastEval"
    default_metric = "SMAPE"
    larger_better = False

    def __init__(self, metric=None, seasonal_window: int = 1, **kw):
        super().__init__(metric, **kw)
        self.seasonal_window = seasonal_window

    def evaluate_arrays(self, y, pred, raw, prob):
        return M.forecast_metrics(pred, y, self.seasonal_window)


class OpLogLossEvaluator(OpEvaluatorBase):
    """``LogLoss`` (OPLogLoss.scala): the mean of -log(probability of the true label); ``binary`` names the
    metric ``BinarylogLoss``, else ``MultiClasslogLoss``."""
    name = "logLoss"
    default_metric = "MultiClasslogLoss"
    larger_better = False

    def __init__(self, metric=None, binary: bool = False, **kw):
        super().__init__(metric or ("BinarylogLoss" if binary else "MultiClasslogLoss"), **kw)

    def evaluate_arrays(self, y, pred, raw, prob):
        return {self.metric: M.log_loss(prob, y)}


class CustomEvaluator(OpEvaluatorBase):
    """``Evaluators.*.custom(metricName, isLargerBetter, evaluateFn)``."""

    def __init__(self, metric_name: str, is_larger_better: bool, fn: Callable, **kw):
        super().__init__(metric_name, **kw)
        self.larger_better = is_larger_better
        self.fn = fn

    def evaluate_arrays(self, y, pred, raw, prob):
        return {self.metric: float(self.fn(y, pred, raw, prob))}


def _custom(metric_name, is_larger_better, evaluate_fn):
    """``Evaluators.*.custom`` (Evaluators.scala:126-140): larger is better unless said otherwise."""
    if evaluate_fn is None:
        raise ValueError("a custom evaluator needs evaluate_fn")
    return CustomEvaluator(metric_name, is_larger_better, evaluate_fn)


class Evaluators:
    """Factory mirroring ``Evaluators.scala``."""

    class BinaryClassification:
        def __new__(cls):
            return OpBinaryClassificationEvaluator()

        @staticmethod
        def auPR():
            return OpBinaryClassificationEvaluator("AuPR")

        @staticmethod
        def auROC():
            return OpBinaryClassificationEvaluator("AuROC")

        @staticmethod
        def precision():
            return OpBinaryClassificationEvaluator("Precision")

        @staticmethod
        def recall():
            return OpBinaryClassificationEvaluator("Recall")

        @staticmethod
        def f1():
            return OpBinaryClassificationEvaluator("F1")

        @staticmethod
        def error():
            return OpBinaryClassificationEvaluator("Error")

        @staticmethod
        def brierScore():
            return OpBinScoreEvaluator("BrierScore")

        @staticmethod
        def custom(metric_name, is_larger_better=True, evaluate_fn=None):
            return _custom(metric_name, is_larger_better, evaluate_fn)

    class MultiClassification:
        def __new__(cls):
            return OpMultiClassificationEvaluator()

        @staticmethod
        def f1():
            return OpMultiClassificationEvaluator("F1")

        @staticmethod
        def precision():
            return OpMultiClassificationEvaluator("Precision")

        @staticmethod
        def recall():
            return OpMultiClassificationEvaluator("Recall")

        @staticmethod
        def error():
            return OpMultiClassificationEvaluator("Error")

        @staticmethod
        def logLoss():
            return OpLogLossEvaluator()

        @staticmethod
        def custom(metric_name, is_larger_better=True, evaluate_fn=None):
            return _custom(metric_name, is_larger_better, evaluate_fn)

    class Regression:
        def __new__(cls):
            return OpRegressionEvaluator()

        @staticmethod
        def rmse():
            return OpRegressionEvaluator("RootMeanSquaredError")

        @staticmethod
        def mse():
            return OpRegressionEvaluator("MeanSquaredError")

        @staticmethod
        def mae():
            return OpRegressionEvaluator("MeanAbsoluteError")

        @staticmethod
        def r2():
            return OpRegressionEvaluator("R2")

        @staticmethod
        def custom(metric_name, is_larger_better=True, evaluate_fn=None):
            return _custom(metric_name, is_larger_better, evaluate_fn)

    class Forecast:
        def __new__(cls):
            return OpForecastEvaluator()

        @staticmethod
        def smape():
            return OpForecastEvaluator("SMAPE")

        @staticmethod
        def mase(seasonal_window=1):
            return OpForecastEvaluator("MASE", seasonal_window)


def evaluator_from_json(d) -> OpEvaluatorBase:
    cls = {c.__name__: c for c in (OpBinaryClassificationEvaluator, OpBinScoreEvaluator,
                                   OpMultiClassificationEvaluator, OpRegressionEvaluator, OpForecastEvaluator,
                                   OpLogLossEvaluator)}[d["className"]]
    return cls(d.get("metric"), uid=d.get("uid"))
