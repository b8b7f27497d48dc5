"""Model selector extras: random hyper-parameter search spaces and two-selector model combination.

Reference: ``RandomParamBuilder`` (``core/.../stages/impl/selector/RandomParamBuilder.scala:52-196``: uniform /
exponential (log-uniform) / subset distributions, ``build(n)``) and ``SelectedModelCombiner`` /
``SelectedCombinerModel`` (``SelectedModelCombiner.scala:72-248``: ``Best`` / ``Weighted`` / ``Equal``
weights from the two selectors' winning validation metrics, weighted raw predictions and
probabilities).
"""
from __future__ import annotations

import math
import random as _random
from typing import Any, Dict, List, Optional, Sequence

import torch

from ..data.columns import PredictionColumn
from ..features import types as T
from ..stages.base import OpEstimator, OpTransformer, register_stage
from .model_selector import SUMMARY_KEY


class RandomParamBuilder:
    """Random search grids: ``RandomParamBuilder(seed).uniform("reg_param", 0, 1).subset(...).build(n)``."""

    def __init__(self, seed: Optional[int] = None):
        self.random = _random.Random(seed)
        self.defs: "Dict[str, tuple]" = {}

    def subset(self, param: str, values: Sequence[Any]) -> "RandomParamBuilder":
        self.defs[param] = ("subset", None, None, list(values))
        return self

    def uniform(self, param: str, lo=None, hi=None) -> "RandomParamBuilder":
        if lo is None and hi is None:          # boolean param
            self.defs[param] = ("uniform_bool", False, True, [])
            return self
        if not lo < hi:
            raise ValueError("Min must be less than max")
        kind = "uniform_int" if isinstance(lo, int) and isinstance(hi, int) else "uniform"
        self.defs[param] = (kind, lo, hi, [])
        return self

    def exponential(self, param: str, lo: float, hi: float) -> "RandomParamBuilder":
        if lo <= 0:
            raise ValueError("Min value must be greater than zero for exponential distribution to work")
        if not lo < hi:
            raise ValueError("Min must be less than max")
        self.defs[param] = ("exponential", lo, hi, [])
        return self

    def build(self, total: int) -> List[Dict[str, Any]]:
        r = self.random
        out = []
        for _ in range(total):
            p = {}
            for name, (kind, lo, hi, seq) in self.defs.items():
                if kind == "subset":
                    p[name] = seq[r.randrange(len(seq))]
                elif kind == "uniform":
                    p[name] = (hi - lo) * r.random() + lo
                elif kind == "uniform_int":
                    p[name] = r.randrange(hi - lo) + lo
                elif kind == "uniform_bool":
                    p[name] = r.random() < 0.5
                else:
                    a, b = math.log10(lo), math.log10(hi)
                    p[name] = 10 ** ((b - a) * r.random() + a)
            out.append(p)
        return out


class CombinationStrategy:
    Best, Weighted, Equal = "best", "weighted", "equal"


def _winning_metric(summary) -> Optional[float]:
    metric = summary.get("evaluationMetric")
    best_params = summary.get("bestModelParameters", {})
    best = summary.get("bestModelName")
    vals = [r["metricValues"].get(metric) for r in summary.get("validationResults", [])
            if r.get("modelName") == best and all(r["modelParameters"].get(k) == v for k, v in best_params.items()
                                                  if k in r["modelParameters"])]
    vals = [v for v in vals if v is not None]
    return max(vals) if vals else None


@register_stage
class SelectedCombinerModel(OpTransformer):
    operation_name = "combineModels"
    output_type = T.Prediction
    arity = 3
    allow_label_as_input = True

    def __init__(self, weight1: float = 0.5, weight2: float = 0.5, strategy: str = "best", metric: str = "",
                 uid=None, **kw):
        super().__init__(uid=uid, **kw)
        self.weight1, self.weight2, self.strategy, self.metric = weight1, weight2, strategy, metric
        self.evaluators = []

    def transform_columns(self, label, p1: PredictionColumn, p2: PredictionColumn, ds=None):
        w1, w2 = self.weight1, self.weight2
        raw = p1.raw * w1 + p2.raw * w2 if p1.raw.shape == p2.raw.shape else p1.raw
        prob = p1.probability * w1 + p2.probability * w2 if p1.probability.shape == p2.probability.shape \
            else p1.probability
        if prob.shape[1] > 0:
            pred = torch.argmax(prob, 1).to(torch.float64)
        else:
            pred = p1.prediction * w1 + p2.prediction * w2
        return PredictionColumn(pred, raw, prob)

    def evaluate_model(self, ds) -> Dict:
        out = self.transform_columns(None, ds[self._inputs[1].name], ds[self._inputs[2].name])
        y = ds[self._inputs[0].name].values.to(torch.float64)
        res = {}
        for ev in self.evaluators:
            res.update(ev.evaluate_arrays(y, out.prediction, out.raw, out.probability))
        if SUMMARY_KEY in self.metadata:
            self.metadata[SUMMARY_KEY]["holdoutEvaluation"] = res
        return res

    def ctor_args(self):
        return {"weight1": self.weight1, "weight2": self.weight2, "strategy": self.strategy, "metric": self.metric}

    def load_ctor_args(self, a):
        self.weight1, self.weight2 = float(a["weight1"]), float(a["weight2"])
        self.strategy, self.metric = a["strategy"], a["metric"]


@register_stage
class SelectedModelCombiner(OpEstimator):
    """(label, prediction of selector 1, prediction of selector 2) -> combined Prediction."""
    operation_name = "combineModels"
    output_type = T.Prediction
    arity = 3
    allow_label_as_input = True
    _defaults = {"combination_strategy": CombinationStrategy.Best}

    def _summaries(self):
        from .model_selector import ModelSelector
        out = []
        for f in self._inputs[1:]:
            st = f.origin_stage
            if not isinstance(st, ModelSelector):
                raise ValueError("Predictions must be from model selectors - other types of model are not supported")
            out.append(st)
        return out

    def fit_columns(self, label, p1, p2, ds=None):
        ms1, ms2 = self._summaries()
        s1, s2 = ms1.metadata.get(SUMMARY_KEY, {}), ms2.metadata.get(SUMMARY_KEY, {})
        if s1.get("problemType") != s2.get("problemType"):
            raise ValueError(f"Cannot combine model selectors for different problem types found "
                             f"{s1.get('problemType')} and {s2.get('problemType')}")
        e1, e2 = s1.get("evaluationMetric"), s2.get("evaluationMetric")
        if e1 == e2:
            m1, m2, metric = _winning_metric(s1), _winning_metric(s2), e1
        else:
            t1, t2 = s1.get("trainEvaluation", {}), s2.get("trainEvaluation", {})
            if e1 in t2:
                m1, m2, metric = t1.get(e1), t2.get(e1), e1
            elif e2 in t1:
                m1, m2, metric = t1.get(e2), t2.get(e2), e2
            else:
                m1 = m2 = None
                metric = e1
        if m1 is None or m2 is None:
            raise RuntimeError("Evaluation metrics for two model selectors are non-overlapping")
        larger = ms1.validator.evaluator.is_larger_better
        strat = str(self.params["combination_strategy"]).lower()
        if strat == CombinationStrategy.Best:
            first = (m1 > m2) == larger
            w1, w2 = (1.0, 0.0) if first else (0.0, 1.0)
        elif strat == CombinationStrategy.Weighted:
            w1, w2 = m1 / (m1 + m2), m2 / (m1 + m2)
        elif strat == CombinationStrategy.Equal:
            w1, w2 = 0.5, 0.5
        else:
            raise ValueError(f"Combination strategy {strat} is not supported")
        model = SelectedCombinerModel(w1, w2, strat, metric)
        evs = list(ms1.evaluators) + [e for e in ms2.evaluators
                                      if type(e) not in {type(x) for x in ms1.evaluators}]
        model.evaluators = evs
        if strat == CombinationStrategy.Best:
            summ = dict(s1 if w1 > 0.5 else s2)
        else:
            out = model.transform_columns(label, p1, p2)
            y = label.values.to(torch.float64)
            train_eval = {}
            for ev in evs:
                train_eval.update(ev.evaluate_arrays(y, out.prediction, out.raw, out.probability))
            summ = {
                "validationType": s1.get("validationType"),
                "validationParameters": {**{k + "_1": v for k, v in s1.get("validationParameters", {}).items()},
                                         **{k + "_2": v for k, v in s2.get("validationParameters", {}).items()}},
                "dataPrepParameters": {**{k + "_1": v for k, v in s1.get("dataPrepParameters", {}).items()},
                                       **{k + "_2": v for k, v in s2.get("dataPrepParameters", {}).items()}},
                "dataPrepResults": s1.get("dataPrepResults") or s2.get("dataPrepResults"),
                "evaluationMetric": metric, "problemType": s1.get("problemType"),
                "bestModelUID": f"{s1.get('bestModelUID')} {s2.get('bestModelUID')}",
                "bestModelName": f"{s1.get('bestModelName')} {s2.get('bestModelName')}",
                "bestModelType": f"{s1.get('bestModelType')} {s2.get('bestModelType')}",
                "validationResults": list(s1.get("validationResults", [])) + list(s2.get("validationResults", [])),
                "trainEvaluation": train_eval, "holdoutEvaluation": None}
        self.metadata[SUMMARY_KEY] = summ
        return model
