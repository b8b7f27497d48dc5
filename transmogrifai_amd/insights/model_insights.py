"""Model insights: label summary, per-raw-feature derived insights, selected model info.

Reference: ``core/.../op/ModelInsights.scala`` -- ``ModelInsights`` (``:74-99``), ``LabelSummary``
(``:293-330``), ``FeatureInsights`` / ``Insights`` (``:338-391``), ``extractFromStages`` (``:444-525``),
``getFeatureInsights`` (``:569-742``) and ``getModelContributions`` (``:784-820``).

Everything here is host-side bookkeeping over already-computed statistics: the SanityChecker summary
(correlations, Cramér's V, moments -- computed by the device column-stat / Gram kernels), the model
selector summary, and the selected learner's feature contributions.
"""
from __future__ import annotations

import json
import math
from collections import OrderedDict
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ..data.vector_metadata import NULL_STRING, OpVectorMetadata

OTHER_STRING = "OTHER"


@dataclass
class LabelSummary:
    labelName: Optional[str] = None
    rawFeatureName: List[str] = field(default_factory=list)
    rawFeatureType: List[str] = field(default_factory=list)
    stagesApplied: List[str] = field(default_factory=list)
    sampleSize: Optional[float] = None
    distribution: Optional[Dict[str, Any]] = None


@dataclass
class Insights:
    derivedFeatureName: str
    stagesApplied: List[str]
    derivedFeatureGroup: Optional[str]
    derivedFeatureValue: Optional[str]
    excluded: Optional[bool] = None
    corr: Optional[float] = None
    cramersV: Optional[float] = None
    mutualInformation: Optional[float] = None
    pointwiseMutualInformation: Dict[str, float] = field(default_factory=dict)
    countMatrix: Dict[str, float] = field(default_factory=dict)
    contribution: List[float] = field(default_factory=list)
    min: Optional[float] = None
    max: Optional[float] = None
    mean: Optional[float] = None
    variance: Optional[float] = None


@dataclass
class FeatureInsights:
    featureName: str
    featureType: str
    derivedFeatures: List[Insights]
    metrics: List[Dict] = field(default_factory=list)
    distributions: List[Dict] = field(default_factory=list)
    exclusionReasons: List[Dict] = field(default_factory=list)
    sensitiveInformation: List[Dict] = field(default_factory=list)


def _clean(v):
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return str(v)
    if isinstance(v, (np.floating, np.integer)):
        return _clean(v.item())
    if isinstance(v, dict):
        return {str(k): _clean(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_clean(x) for x in v]
    if isinstance(v, np.ndarray):
        return _clean(v.tolist())
    return v


@dataclass
class ModelInsights:
    label: LabelSummary
    features: List[FeatureInsights]
    selectedModelInfo: Optional[Dict[str, Any]]
    trainingParams: Dict[str, Any]
    stageInfo: Dict[str, Any]

    def to_json_dict(self) -> Dict[str, Any]:
        return _clean(asdict(self))

    def to_json(self, pretty: bool = True) -> str:
        return json.dumps(self.to_json_dict(), indent=2 if pretty else None)

    @staticmethod
    def from_json(s: str) -> "ModelInsights":
        d = json.loads(s) if isinstance(s, str) else s
        feats = [FeatureInsights(f["featureName"], f["featureType"],
                                 [Insights(**i) for i in f.get("derivedFeatures", [])],
                                 f.get("metrics", []), f.get("distributions", []), f.get("exclusionReasons", []),
                                 f.get("sensitiveInformation", [])) for f in d.get("features", [])]
        return ModelInsights(LabelSummary(**d.get("label", {})), feats, d.get("selectedModelInfo"),
                             d.get("trainingParams", {}), d.get("stageInfo", {}))

    def pretty_print(self, top_k: int = 15) -> str:
        from .pretty import pretty_insights
        return pretty_insights(self, top_k)


# ------------------------------------------------------------------------------------------ extraction
def _find_selector(model, pred_feature):
    from ..selector.model_selector import SelectedModel
    if pred_feature is not None:
        for st in model.stages:
            if st.uid == pred_feature.origin_stage.uid:
                return st
    return next((st for st in model.stages if isinstance(st, SelectedModel)), None)


def _vector_meta_of(model, feature) -> Optional[OpVectorMetadata]:
    st = next((s for s in model.stages if s.uid == feature.origin_stage.uid), None)
    if st is None:
        return None
    return st.metadata.get("vector_metadata")


def _sanity_summary(model, feature):
    from ..stages.preparators.sanity_checker import SanityCheckerModel
    st = next((s for s in model.stages if s.uid == feature.origin_stage.uid), None)
    if isinstance(st, SanityCheckerModel):
        return st, st.metadata.get("summary")
    return None, None


def _label_summary(model, label_feature, sanity) -> LabelSummary:
    if label_feature is None:
        return LabelSummary()
    hist = label_feature.history()
    raw = label_feature.raw_features()
    ls = LabelSummary(labelName=label_feature.name, rawFeatureName=[f.name for f in raw],
                      rawFeatureType=[f.type_name for f in raw], stagesApplied=list(hist.stages))
    if sanity is not None:
        fs = sanity.get("featuresStatistics", {})
        ls.sampleSize = fs.get("count")
        labs = [s for s in sanity.get("categoricalStats", [])]
        cs = next((c for c in sanity.get("columnStatistics", []) if c.get("isLabel")), None)
        if cs is not None:
            ls.distribution = {"type": "Continuous", "min": cs["min"], "max": cs["max"], "mean": cs["mean"],
                               "variance": cs["variance"]}
        dist = sanity.get("labelDistribution")
        if dist is not None:
            ls.distribution = {"type": "Discrete", "domain": dist["domain"], "prob": dist["prob"]}
        del labs
    return ls


def _contributions(selected, d: int) -> Optional[np.ndarray]:
    if selected is None:
        return None
    try:
        c = selected.learner.feature_contributions(selected.state, d)
    except Exception:   # a learner without contributions
        return None
    if c is None:
        return None
    c = np.asarray(c, np.float64)
    if c.ndim == 1:
        c = c[None, :]
    return c


def extract_model_insights(model, pred_feature=None) -> ModelInsights:
    """Build :class:`ModelInsights` from a fitted workflow model (``ModelInsights.extractFromStages``)."""
    selected = _find_selector(model, pred_feature)
    label_feature = None
    vec_feature = None
    if selected is not None and len(selected._inputs) == 2:
        label_feature, vec_feature = selected._inputs
    sc_stage, sanity = (None, None)
    model_meta = None
    if vec_feature is not None:
        sc_stage, sanity = _sanity_summary(model, vec_feature)
        model_meta = _vector_meta_of(model, vec_feature)
    # full (pre-sanity-checker) metadata: all derived columns, with dropped ones marked excluded
    full_meta = None
    if sc_stage is not None:
        full_meta = _vector_meta_of(model, sc_stage._inputs[1])
    all_meta = full_meta or model_meta
    stats_by_name: Dict[str, Dict] = {}
    cat_by_name: Dict[str, Dict] = {}
    dropped = set()
    if sanity is not None:
        for s in sanity.get("columnStatistics", []):
            stats_by_name[s["name"]] = s
        for g in sanity.get("categoricalStats", []):
            for k, f in enumerate(g.get("categoricalFeatures", [])):
                cat_by_name[f] = dict(g, _pos=k)
        dropped = set(sanity.get("dropped", []))
    contrib = None
    kept_pos: Dict[int, int] = {}          # column index in all_meta -> column of the model's input
    if model_meta is not None:
        contrib = _contributions(selected, model_meta.size)
        if sc_stage is not None and full_meta is not None and sc_stage.remove_bad_features:
            kept_pos = {int(i): k for k, i in enumerate(sc_stage.indices_to_keep)}
        else:
            kept_pos = {i: i for i in range(model_meta.size)}
    feats: "OrderedDict[str, FeatureInsights]" = OrderedDict()
    raw_types: Dict[str, str] = {}
    for f in model.raw_features:
        raw_types[f.name] = f.type_name
    if all_meta is not None:
        hist = all_meta.history
        for c in all_meta.columns:
            name = c.make_col_name()
            st = stats_by_name.get(name, {})
            cat = cat_by_name.get(name)
            ins = Insights(
                derivedFeatureName=name,
                stagesApplied=sorted({s for p in c.parent_feature_name
                                      for s in (hist[p].stages if p in hist else ())}),
                derivedFeatureGroup=c.grouping,
                derivedFeatureValue=c.indicator_value if c.indicator_value is not None else c.descriptor_value,
                excluded=(name in dropped) if sanity is not None else None,
                corr=st.get("corrLabel"),
                cramersV=None if cat is None else cat.get("cramersV"),
                mutualInformation=None if cat is None else cat.get("mutualInfo"),
                pointwiseMutualInformation={} if cat is None else _pmi_of(cat),
                countMatrix={} if cat is None else _counts_of(cat),
                contribution=[] if contrib is None or c.index not in kept_pos else
                [float(v) for v in contrib[:, kept_pos[c.index]]],
                min=st.get("min"), max=st.get("max"), mean=st.get("mean"), variance=st.get("variance"))
            origins = []
            for p in c.parent_feature_name:
                origins.extend(hist[p].origin_features if p in hist else (p,))
            for o in dict.fromkeys(origins):
                fi = feats.get(o)
                if fi is None:
                    fi = feats[o] = FeatureInsights(o, raw_types.get(o, c.parent_feature_type[0]), [])
                fi.derivedFeatures.append(ins)
    rff = getattr(model, "raw_feature_filter_results", None)
    if rff is not None and hasattr(rff, "to_json"):
        rff = rff.to_json()
    if rff:
        for m in rff.get("rawFeatureFilterMetrics", []):
            n = m.get("name")
            if n in feats:
                feats[n].metrics.append(m)
        for r in rff.get("exclusionReasons", []):
            n = r.get("name")
            if n in feats:
                feats[n].exclusionReasons.append(r)
        for dd in rff.get("rawFeatureDistributions", []):
            n = dd.get("name")
            if n in feats:
                feats[n].distributions.append(dd)
    label = _label_summary(model, label_feature, sanity)
    sel_info = selected.metadata.get("summary") if selected is not None else None
    stage_info = OrderedDict()
    for st in model.stages:
        stage_info[st.uid] = {"stageName": type(st).__name__, "uid": st.uid,
                              "params": {k: _clean(v) for k, v in st.params.items() if _jsonable(v)}}
    params = model.parameters.to_json() if hasattr(model.parameters, "to_json") else {}
    return ModelInsights(label, list(feats.values()), sel_info, params, stage_info)


def _jsonable(v) -> bool:
    return isinstance(v, (int, float, str, bool, type(None), list, tuple, dict))


def _per_label(cat, key) -> Dict[str, float]:
    """``{label: value}`` for this column's row of a ``{label: [row values]}`` contingency-shaped map."""
    m = cat.get(key)
    if not m:
        return {}
    k = cat["_pos"]
    labels = cat.get("labels")
    out = {}
    for j, vals in m.items():
        if k < len(vals):
            name = labels[int(j)] if labels is not None and int(j) < len(labels) else j
            out[str(name)] = float(vals[k])
    return out


def _pmi_of(cat) -> Dict[str, float]:
    return _per_label(cat, "pmi")


def _counts_of(cat) -> Dict[str, float]:
    return _per_label(cat, "contingency")
