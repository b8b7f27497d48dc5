"""Human-readable model summary (``ModelInsights.prettyPrint``, ``ModelInsights.scala:101-290``;
``OpWorkflowModel.summaryPretty``, ``OpWorkflowModel.scala:206-215``)."""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

from ..data.vector_metadata import NULL_STRING
from ..utils.table import pretty_table

OTHER_STRING = "OTHER"

_NICE_METRICS = {"AuROC": "area under ROC", "AuPR": "area under precision-recall", "Precision": "precision",
                 "Recall": "recall", "F1": "f1 score", "Error": "error rate", "TP": "true positive",
                 "TN": "true negative", "FP": "false positive", "FN": "false negative",
                 "RootMeanSquaredError": "root mean square error", "MeanSquaredError": "mean square error",
                 "R2": "r2", "MeanAbsoluteError": "mean absolute error", "BrierScore": "brier score",
                 "LogLoss": "log loss"}

_VALIDATION_NAMES = {"CrossValidation": "Cross Validation", "TrainValidationSplit": "Train Validation Split"}

_EXCLUDED_PARAMS = {"inputFeatures", "inputSchema", "outputMetadata", "labelCol", "predictionCol",
                    "predictionValueCol", "rawPredictionCol", "probabilityCol"}


def _nice(metric: str) -> str:
    return _NICE_METRICS.get(metric.split("_")[-1], metric)


def _validation_results(info) -> List[str]:
    if not info:
        return ["No model selector found"]
    vr = info.get("validationResults", [])
    types = list(dict.fromkeys(v["modelType"] for v in vr))
    metric = info.get("evaluationMetric", "")
    head = "Evaluated %s model%s using %s and %s metric." % (
        ", ".join(types), "s" if len(types) > 1 else "",
        _VALIDATION_NAMES.get(info.get("validationType"), info.get("validationType")), _nice(metric))
    lines = []
    for t in types:
        vals = [float(v["metricValues"][metric]) for v in vr if v["modelType"] == t and metric in v["metricValues"]]
        lo = min(vals) if vals else float("nan")
        hi = max(vals) if vals else float("nan")
        lines.append("Evaluated %d %s model%s with %s metric between [%r, %r]." % (
            len(vals), t, "s" if len(vals) > 1 else "", _nice(metric), lo, hi))
    return [head, "\n".join(lines)]


def _selected_model(info) -> List[str]:
    if not info:
        return []
    params = info.get("bestModelParameters", {}) or {}
    rows = [("name", info.get("bestModelName")), ("uid", info.get("bestModelUID")),
            ("modelType", info.get("bestModelType"))]
    rows += [(k, v) for k, v in params.items() if k not in _EXCLUDED_PARAMS]
    rows.sort(key=lambda r: r[0])
    return [pretty_table(["Model Param", "Value"], rows, name=f"Selected Model - {info.get('bestModelType')}")]


def _flat_metrics(m) -> dict:
    out = {}
    for k, v in (m or {}).items():
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            out[k] = float(v)
    return out


def _evaluation_metrics(info) -> List[str]:
    if not info:
        return []
    tr = _flat_metrics(info.get("trainEvaluation"))
    ho = info.get("holdoutEvaluation")
    if tr and ho:
        hf = _flat_metrics(ho)
        rows = sorted((_nice(k), repr(v), repr(hf.get(k, float("nan")))) for k, v in tr.items())
        return [pretty_table(["Metric Name", "Training Set Value", "Hold Out Set Value"], rows,
                             name="Model Evaluation Metrics")]
    if tr:
        rows = sorted((_nice(k), repr(v)) for k, v in tr.items())
        return [pretty_table(["Metric Name", "Training Set Value"], rows, name="Model Evaluation Metrics")]
    return []


def _derived_non_excluded(mi):
    for f in mi.features:
        for d in f.derivedFeatures:
            if d.excluded is not True:
                yield f, d


def _insight_name(f, d) -> str:
    g, v = d.derivedFeatureGroup, d.derivedFeatureValue
    if g is not None and v == NULL_STRING:
        return f"{f.featureName}({g} = null)"
    if g is not None and v == OTHER_STRING:
        return f"{f.featureName}({g} = other)"
    if g is not None and v is not None:
        return f"{f.featureName}({g} = {v})"
    if g is not None:
        return f"{f.featureName}(group = {g})"
    if v is not None:
        return f"{f.featureName}(value = {v})"
    return f.featureName


def _top_k(items: Sequence[Tuple], k: int) -> List[Tuple[str, float]]:
    out: List[Tuple[str, float]] = []
    seen = set()
    for f, d, val in items:
        name = _insight_name(f, d)
        if name in seen:
            continue
        seen.add(name)
        out.append((name, val))
        if len(out) >= k:
            break
    return out


def _num(v):
    return v is not None and not (isinstance(v, float) and math.isnan(v))


def _correlations(mi, k) -> List[str]:
    items = [(f, d, d.corr if _num(d.corr) else None) for f, d in _derived_non_excluded(mi)]
    dsc = sorted(items, key=lambda t: t[2] if t[2] is not None else -math.inf, reverse=True)
    asc = sorted(items, key=lambda t: t[2] if t[2] is not None else math.inf)
    pos = _top_k([t for t in dsc if t[2] is not None], k)
    neg = [r for r in _top_k([t for t in asc if t[2] is not None], k) if r not in pos]
    col = "Correlation Value"
    out = [pretty_table(["Top Positive Correlations", col], pos, name="Top Model Insights")]
    if neg:
        out.append(pretty_table(["Top Negative Correlations", col], neg))
    return out


def _contributions(mi, k) -> List[str]:
    items = [(f, d, abs(max(d.contribution)) if d.contribution else 0.0) for f, d in _derived_non_excluded(mi)]
    items.sort(key=lambda t: t[2], reverse=True)
    rows = _top_k(items, k)
    return [pretty_table(["Top Contributions", "Contribution Value"], rows)] if rows else []


def _cramers_v(mi, k) -> List[str]:
    rows = []
    for f, d in _derived_non_excluded(mi):
        if d.derivedFeatureGroup is not None and _num(d.cramersV):
            r = (d.derivedFeatureGroup, d.cramersV)
            if r not in rows:
                rows.append(r)
    rows.sort(key=lambda r: r[1], reverse=True)
    rows = rows[:k]
    return [pretty_table(["Top CramersV", "CramersV"], rows)] if rows else []


def pretty_insights(mi, top_k: int = 15) -> str:
    info = mi.selectedModelInfo
    parts: List[str] = []
    parts += _validation_results(info)
    parts += _selected_model(info)
    parts += _evaluation_metrics(info)
    parts += _correlations(mi, top_k)
    parts += _contributions(mi, top_k)
    parts += _cramers_v(mi, top_k)
    return "\n".join(parts)


def summary_pretty(model, top_k: int = 15) -> str:
    return model.model_insights().pretty_print(top_k)
