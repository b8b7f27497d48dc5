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
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):     # Java's Double.toString spellings
        return "NaN" if math.isnan(v) else ("Infinity" if v > 0 else "-Infinity")
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
        d = _clean(asdict(self))
        for f in d.get("features", []):        # cardinality estimates stay in memory (FeatureDistribution JSON)
            for x in f.get("distributions", []):
                x.pop("cardEstimate", None)
        return d

    def to_json(self, pretty: bool = True) -> str:
        return json.dumps(self.to_json_dict(), indent=2 if pretty else None)

    @staticmethod
    def from_json(s: str) -> "ModelInsights":
        d = json.loads(s) if isinstance(s, str) else s
        feats = [FeatureInsights(f["featureName"], f["featureType"],
                                 [Insights(**_unclean_insights(i)) for i in f.get("derivedFeatures", [])],
                                 f.get("metrics", []), f.get("distributions", []), f.get("exclusionReasons", []),
                                 f.get("sensitiveInformation", [])) for f in d.get("features", [])]
        return ModelInsights(LabelSummary(**d.get("label", {})), feats, d.get("selectedModelInfo"),
                             d.get("trainingParams", {}), d.get("stageInfo", {}))

    def pretty_print(self, top_k: int = 15) -> str:
        from .pretty import pretty_insights
        return pretty_insights(self, top_k)


_NONFINITE = {"NaN": float("nan"), "nan": float("nan"), "Infinity": float("inf"), "inf": float("inf"),
              "-Infinity": float("-inf"), "-inf": float("-inf")}


def _unclean_insights(i: Dict) -> Dict:
    """The numeric fields of a serialised :class:`Insights` back to floats (non-finite values travel as strings)."""
    out = dict(i)
    for k in ("corr", "cramersV", "mutualInformation", "min", "max", "mean", "variance"):
        v = out.get(k)
        if isinstance(v, str) and v in _NONFINITE:
            out[k] = _NONFINITE[v]
    for k in ("pointwiseMutualInformation", "countMatrix"):
        if isinstance(out.get(k), dict):
            out[k] = {a: _NONFINITE.get(b, b) if isinstance(b, str) else b for a, b in out[k].items()}
    if isinstance(out.get("contribution"), list):
        out["contribution"] = [_NONFINITE.get(b, b) if isinstance(b, str) else b for b in out["contribution"]]
    return out


# ------------------------------------------------------------------------------------------ extraction
def _is_model_stage(st) -> bool:
    from ..models.base import OpPredictorModel
    from ..selector.extras import SelectedCombinerModel
    return isinstance(st, (OpPredictorModel, SelectedCombinerModel))


def _upstream_uids(feature) -> set:
    """uids of every stage that feature depends on, its origin stage included (``FeatureLike.parentStages``)."""
    return {st.uid for st in feature.parent_stages()}


def _vector_meta_of(model, feature) -> Optional[OpVectorMetadata]:
    st = next((s for s in model.stages if s.uid == feature.origin_stage.uid), None)
    if st is None:
        return None
    return st.metadata.get("vector_metadata")


def _flatten_summaries(summaries: Sequence[Dict]) -> Optional[Dict]:
    """``SanityCheckerSummary.flatten`` (SanityCheckerMetadata.scala:337-344): list fields concatenated, the first
    checker's count and sample fraction."""
    summaries = [x for x in summaries if x]
    if not summaries:
        return None
    if len(summaries) == 1:
        return summaries[0]
    first = summaries[0]
    fs0 = first.get("featuresStatistics", {})
    fs = {"count": fs0.get("count"), "sampleFraction": fs0.get("sampleFraction")}
    for k in ("min", "max", "mean", "variance"):
        fs[k] = [v for x in summaries for v in x.get("featuresStatistics", {}).get(k, [])]
    corr = {"featuresIn": [v for x in summaries for v in x.get("correlationsWLabel", {}).get("featuresIn", [])],
            "values": [v for x in summaries for v in x.get("correlationsWLabel", {}).get("values", [])],
            "correlationType": first.get("correlationsWLabel", {}).get("correlationType")}
    return {"names": [v for x in summaries for v in x.get("names", [])],
            "featuresStatistics": fs, "correlationsWLabel": corr,
            "dropped": [v for x in summaries for v in x.get("dropped", [])],
            "categoricalStats": [v for x in summaries for v in x.get("categoricalStats", [])],
            "labelDistribution": summaries[-1].get("labelDistribution")}


def get_label_summary(label_feature, summary: Optional[Dict]) -> LabelSummary:
    """``ModelInsights.getLabelSummary`` (ModelInsights.scala:534-568): the label's history, and from the sanity
    checker summary the sample size and the distribution -- Discrete (domain / probabilities from the first
    contingency matrix's label sums) when there are categorical statistics, else Continuous (the label's
    moments, the last entry of the feature statistics)."""
    if label_feature is None:
        return LabelSummary()
    hist = label_feature.history()
    raw = label_feature.raw_features()
    ls = LabelSummary(labelName=label_feature.name, rawFeatureName=list(hist.origin_features),
                      rawFeatureType=[f.type_name for f in raw], stagesApplied=list(hist.stages))
    if summary is not None:
        fs = summary.get("featuresStatistics", {})
        ls.sampleSize = fs.get("count")
        cats = summary.get("categoricalStats") or []
        if not cats:
            last = (lambda k: (fs.get(k) or [None])[-1])
            ls.distribution = {"type": "Continuous", "min": last("min"), "max": last("max"), "mean": last("mean"),
                               "variance": last("variance")}
        else:
            cm = cats[0].get("contingencyMatrix") or cats[0].get("contingency") or {}
            labels = cats[0].get("labels")
            counts = sorted(((str(labels[int(k)]) if labels is not None and str(k).isdigit() and int(k) < len(labels)
                              else str(k)), float(sum(v))) for k, v in cm.items())
            total = sum(c for _, c in counts)
            ls.distribution = {"type": "Discrete", "domain": [k for k, _ in counts],
                               "prob": [c / total if total else 0.0 for _, c in counts]}
    return ls


def _label_std(label: LabelSummary) -> float:
    """Standard deviation of the label for LinearRegression descaling (ModelInsights.scala:600-632); 1.0 when
    unknown, unsupported or zero."""
    d = label.distribution
    if not d:
        return 1.0
    if d.get("type") == "Continuous":
        v = d.get("variance")
        return math.sqrt(v) if v else 1.0
    if d.get("type") == "Discrete":
        try:
            dom = [float(x) for x in d["domain"]]
        except (TypeError, ValueError):
            return 1.0
        prob = d["prob"]
        mean = sum(x * p for x, p in zip(dom, prob))
        var = sum((x - mean) ** 2 * p for x, p in zip(dom, prob))
        return math.sqrt(var) if var else 1.0
    return 1.0


def get_model_contributions(model_stage, d: Optional[int] = None) -> List[List[float]]:
    """``ModelInsights.getModelContributions`` (ModelInsights.scala:784-830): one list per coefficient row (the
    multinomial LR / NaiveBayes matrices have one per class), feature importances of the tree ensembles, nothing for
    models without contributions (the model combiner, MLP)."""
    if model_stage is None or not hasattr(model_stage, "learner_name") or model_stage.state is None:
        return []
    size = d if d is not None else _input_size(model_stage)
    try:
        c = model_stage.learner.feature_contributions(model_stage.state, size)
    except Exception:   # noqa: BLE001 - a learner without contributions
        return []
    if c is None:
        return []
    c = np.asarray(c, np.float64)
    if c.ndim == 1:
        c = c[None, :]
    return [list(map(float, row)) for row in c]


def _input_size(model_stage) -> int:
    st = model_stage.state or {}
    for k in ("coefficients", "coefficient_matrix"):
        if k in st:
            return int(np.asarray(st[k]).shape[-1])
    return int(st.get("n_features", 0) or 0)


def descale_lr_contrib(model_stage, contrib: Sequence[float], feature_std: float, label_std: float) -> List[float]:
    """``ModelInsights.descaleLRContrib`` (ModelInsights.scala:754-782): with standardization on, a logistic
    regression's coefficients are reported as standardized coefficients (times the feature's standard deviation;
    Agresti 4.5.2) and a linear regression's also divided by the label's standard deviation."""
    name = getattr(model_stage, "learner_name", None)
    params = getattr(model_stage, "learner_params", {}) or {}
    if not contrib or not params.get("standardization", False):
        return list(contrib)
    if name == "OpLogisticRegression":
        return [c * feature_std for c in contrib]
    if name == "OpLinearRegression":
        return [c * feature_std / label_std for c in contrib]
    return list(contrib)


def get_feature_insights(meta: Optional[OpVectorMetadata], summary: Optional[Dict], model_stage,
                         raw_features: Sequence = (), blocklisted: Sequence = (),
                         blocklisted_map_keys: Optional[Dict[str, Sequence[str]]] = None, rff_results=None,
                         label: Optional[LabelSummary] = None) -> List[FeatureInsights]:
    """``ModelInsights.getFeatureInsights`` (ModelInsights.scala:569-742): one :class:`Insights` per derived column of
    the feature vector, grouped under every raw feature it originates from, plus the blocklisted raw features and map
    keys (``excluded = true``), the raw feature filter's metrics / distributions / exclusion reasons per raw feature,
    and the vector's sensitive-feature information."""
    label = label or LabelSummary()
    pairs: List[tuple] = []         # (origin raw feature names, Insights)
    if meta is not None and summary is not None:
        contributions = get_model_contributions(model_stage, meta.size)
        dropped = set(summary.get("dropped", []))
        kept = {c.index: k for k, c in enumerate(c for c in meta.columns if c.make_col_name() not in dropped)}
        fs = summary.get("featuresStatistics", {})
        pos = {}
        for i, n in enumerate(summary.get("names", [])):
            pos.setdefault(n, i)
        cw = summary.get("correlationsWLabel", {})
        corr_pos = {}
        for i, n in enumerate(cw.get("featuresIn", [])):
            corr_pos.setdefault(n, i)
        corr_vals = cw.get("values", [])
        cats = summary.get("categoricalStats") or []
        lstd = _label_std(label)
        for h in meta.column_history():
            name = h["columnName"]
            gi = next((k for k, g in enumerate(cats) if name in g.get("categoricalFeatures", [])), None)
            cat = None if gi is None else dict(cats[gi], _pos=cats[gi]["categoricalFeatures"].index(name))
            i = pos[name] if name in pos else (h["index"] if h["index"] < len(fs.get("variance", [])) else None)

            def stat(k, i=i):
                vals = fs.get(k) or []
                return None if i is None or i >= len(vals) else vals[i]
            var = stat("variance")
            fstd = math.sqrt(var) if var is not None and var >= 0 else 1.0
            ki = kept.get(h["index"])
            raw_c = [] if ki is None else [row[ki] if ki < len(row) else 0.0 for row in contributions]
            ci = corr_pos.get(name)
            corr = None
            if ci is not None and ci < len(corr_vals):
                corr = float("nan") if corr_vals[ci] is None else corr_vals[ci]
            pairs.append((h["parentFeatureOrigins"], Insights(
                derivedFeatureName=name, stagesApplied=list(h["parentFeatureStages"]),
                derivedFeatureGroup=h["grouping"],
                derivedFeatureValue=h["indicatorValue"] if h["indicatorValue"] is not None else h["descriptorValue"],
                excluded=name in dropped, corr=corr,
                cramersV=None if cat is None else cat.get("cramersV"),
                mutualInformation=None if cat is None else cat.get("mutualInfo"),
                pointwiseMutualInformation={} if cat is None else _pmi_of(cat),
                countMatrix={} if cat is None else _counts_of(cat),
                contribution=descale_lr_contrib(model_stage, raw_c, fstd, lstd),
                min=stat("min"), max=stat("max"), mean=stat("mean"), variance=var)))
    elif meta is not None:
        contributions = get_model_contributions(model_stage, meta.size)
        for h in meta.column_history():     # nothing dropped without a sanity checker
            pairs.append((h["parentFeatureOrigins"], Insights(
                derivedFeatureName=h["columnName"], stagesApplied=list(h["parentFeatureStages"]),
                derivedFeatureGroup=h["grouping"], derivedFeatureValue=h["indicatorValue"],
                contribution=[row[h["index"]] if h["index"] < len(row) else 0.0 for row in contributions])))
    for f in blocklisted:
        pairs.append(([f.name], Insights(derivedFeatureName=f.name, stagesApplied=[], derivedFeatureGroup=None,
                                         derivedFeatureValue=None, excluded=True)))
    for mname, keys in (blocklisted_map_keys or {}).items():
        for key in keys:
            pairs.append(([mname], Insights(derivedFeatureName=key, stagesApplied=[], derivedFeatureGroup=key,
                                            derivedFeatureValue=None, excluded=True)))
    all_types = {f.name: f.type_name for f in list(raw_features) + list(blocklisted)}
    rff = rff_results.to_json() if rff_results is not None and hasattr(rff_results, "to_json") else \
        (rff_results or {})
    if hasattr(rff_results, "rawFeatureDistributions"):      # in memory: with the cardinality estimates
        rff = dict(rff, rawFeatureDistributions=[d.to_json(with_card=True)
                                                 for d in rff_results.rawFeatureDistributions])
    sens = meta.sensitive if meta is not None else {}

    def new_fi(fname, derived):
        return FeatureInsights(
            featureName=fname, featureType=all_types.get(fname, ""), derivedFeatures=derived,
            metrics=[m for m in rff.get("rawFeatureFilterMetrics", []) if m.get("name") == fname],
            distributions=[d for d in rff.get("rawFeatureDistributions", []) if d.get("name") == fname],
            exclusionReasons=[r for r in rff.get("exclusionReasons", []) if r.get("name") == fname],
            sensitiveInformation=list(sens.get(fname, [])))
    out: "OrderedDict[str, FeatureInsights]" = OrderedDict()
    for origins, ins in pairs:
        for o in dict.fromkeys(origins):
            if o not in out:
                out[o] = new_fi(o, [])
            out[o].derivedFeatures.append(ins)
    # removed sensitive features with no column left in the vector (every action taken)
    for fname, infos in sens.items():
        if fname not in out and infos and all(_get(i, "actionTaken") for i in infos):
            out[fname] = new_fi(fname, [])
    return list(out.values())


def _get(info, key):
    return info.get(key) if isinstance(info, dict) else getattr(info, key, None)


def _stage_info(stages, rff_results=None) -> "OrderedDict[str, Any]":
    """``stageInfo``: the raw feature filter's configuration (when it ran) and every stage's uid and parameters,
    keyed by stage name (``RawFeatureFilterResults.toStageInfo``, ``ModelInsights.getStageInfo``)."""
    info: "OrderedDict[str, Any]" = OrderedDict()
    cfg = getattr(rff_results, "rawFeatureFilterConfig", None) if rff_results is not None else None
    if cfg is not None:
        info["rawFeatureFilter"] = {"uid": "rawFeatureFilter", "params": {k: str(v) for k, v in
                                                                        dict(cfg.__dict__).items()}}
    for st in stages:
        info[st.stage_name()] = {"stageName": type(st).__name__, "uid": st.uid,
                                 "params": {k: _clean(v) for k, v in st.params.items() if _jsonable(v)}}
    return info


def extract_from_stages(stages: Sequence, raw_features: Sequence, training_params: Dict, blocklisted: Sequence = (),
                        blocklisted_map_keys: Optional[Dict[str, Sequence[str]]] = None,
                        rff_results=None, model=None) -> ModelInsights:
    """``ModelInsights.extractFromStages`` (ModelInsights.scala:444-532) over the fitted stages a feature depends
    on: the last model among them (a best-strategy model combiner resolves to its winner), the sanity checkers on
    that model's input path with the same label (else the last one), the label, and the feature vector's metadata --
    the sanity checker's input vector, else the model's input vector, else the last vector-valued stage."""
    from ..stages.preparators.sanity_checker import SanityCheckerModel
    from ..selector.extras import SelectedCombinerModel
    models = [st for st in stages if _is_model_stage(st)]
    resolved = []
    for st in models:
        if isinstance(st, SelectedCombinerModel) and str(st.strategy).lower() == "best":
            origin = st._inputs[1] if st.weight1 > 0.5 else st._inputs[2]
            m = next((x for x in models if x.uid == origin.origin_stage.uid), None)
            if m is not None:
                resolved.append(m)
        else:
            resolved.append(st)
    sel = resolved[-1] if resolved else None
    model_in = set()
    if sel is not None:
        for f in sel._inputs:
            if not f.is_raw:
                model_in |= _upstream_uids(f)
    checkers = [st for st in stages if isinstance(st, SanityCheckerModel)]
    for_model = [c for c in checkers if c.uid in model_in and sel is not None and sel._inputs and
                 c._inputs and sel._inputs[0].uid == c._inputs[0].uid]
    chosen = for_model or checkers[-1:]
    summary = _flatten_summaries([c.metadata.get("summary") for c in chosen])
    label_feature = None
    if sel is not None and sel._inputs:
        label_feature = sel._inputs[0]
    elif chosen:
        label_feature = chosen[-1]._inputs[0]
    by_uid = {st.uid: st for st in stages}

    def meta_of(feature):
        st = by_uid.get(feature.origin_stage.uid) if feature.origin_stage is not None else None
        if st is None and model is not None:
            st = next((s for s in model.stages if s.uid == feature.origin_stage.uid), None)
        return None if st is None else st.metadata.get("vector_metadata")
    meta = None
    if chosen:
        metas = [meta_of(c._inputs[1]) for c in chosen]
        metas = [m for m in metas if m is not None]
        if metas:
            meta = metas[0] if len(metas) == 1 else OpVectorMetadata.flatten("", metas)
    elif sel is not None and len(sel._inputs) == 2:
        meta = meta_of(sel._inputs[1])
    if meta is None and not chosen and sel is None:
        vec = [st for st in stages if isinstance(st.metadata.get("vector_metadata"), OpVectorMetadata)]
        meta = vec[-1].metadata["vector_metadata"] if vec else None
    label = get_label_summary(label_feature, summary)
    feats = get_feature_insights(meta, summary, sel, raw_features, blocklisted, blocklisted_map_keys, rff_results,
                                 label)
    info = sel.metadata.get("summary") if sel is not None else None
    return ModelInsights(label, feats, info, training_params, _stage_info(stages, rff_results))


def extract_model_insights(model, feature=None) -> ModelInsights:
    """Build :class:`ModelInsights` for ``feature`` of a fitted workflow model (``OpWorkflowModel.modelInsights``,
    OpWorkflowModel.scala:198-216): the insights of the stages that feature depends on. A raw feature, or one not
    produced by this model, is an error."""
    if feature is None:
        feature = next((f for f in model.result_features if f.wtype.__name__ == "Prediction"), None)
    if feature is None:
        raise ValueError("No prediction feature in the workflow model: name the feature to get insights on")
    uids = {st.uid for st in model.stages}
    if feature.is_raw or feature.origin_stage is None or feature.origin_stage.uid not in uids:
        raise ValueError(f"Feature '{feature.name}' is either a raw feature or not part of this workflow model")
    up = _upstream_uids(feature)
    stages = [st for st in model.stages if st.uid in up]
    params = model.parameters.to_json() if hasattr(model.parameters, "to_json") else {}
    return extract_from_stages(stages, list(model.raw_features), params, list(getattr(model, "blocklist", [])),
                               dict(getattr(model, "blocklist_map_keys", {}) or {}),
                               getattr(model, "raw_feature_filter_results", None), model)


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
    return _per_label(cat, "contingencyMatrix" if cat.get("contingencyMatrix") else "contingency")
