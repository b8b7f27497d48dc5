"""Model checkpoint writer / reader: the ``op-model.json`` format.

Reference: ``OpWorkflowModelWriter`` (``core/.../OpWorkflowModelWriter.scala:58-183``: fields uid,
resultFeaturesUids, blocklisted*, stages, allFeatures, parameters, trainParameters,
rawFeatureFilterResults; written gzip-compressed as ``op-model.json/part-00000.gz``), the stage writer
(``features/.../stages/OpPipelineStageWriter.scala:67-88``: class, uid, paramMap, ctorArgs) and
``OpWorkflowModelReader`` (``OpWorkflowModelReader.scala:97-266``: falls back through ``part-00000.gz``,
``part-00000`` and the raw path; accepts the legacy ``blacklisted*`` field names). Learned tensors are
stored inline as base64 arrays (:mod:`transmogrifai_amd.utils.serde`); nothing is unpickled on load, and
user functions named by a checkpoint (extract functions) resolve only through the in-process registry
(``stages/generator.py`` ``register_function``): loading never imports a module.
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import time
from typing import Dict, List, Optional

from ..data.vector_metadata import OpVectorMetadata
from ..features import types as T
from ..features.feature import FeatureLike, TransientFeature
from ..stages.base import OpPipelineStage, stage_class
from ..stages.generator import FeatureGeneratorStage
from ..utils.serde import decode, encode
from .params import OpParams

MODEL_DIR = "op-model.json"
PART = "part-00000"


# RawFeatureFilterResults of a workflow trained without a raw feature filter (the reference's defaults,
# RawFeatureFilterResults.scala / OldModelVersion_0_7_1 fixture)
_EMPTY_RFF = {"rawFeatureFilterConfig": {"minFill": 0.0, "maxFillDifference": float("inf"),
                                         "maxFillRatioDiff": float("inf"), "maxJSDivergence": 1.0,
                                         "maxCorrelation": 1.0, "correlationType": "Pearson",
                                         "jsDivergenceProtectedFeatures": [], "protectedFeatures": []},
              "rawFeatureDistributions": [], "rawFeatureFilterMetrics": [], "exclusionReasons": []}

_VECTOR_KEYS = ("vector_columns", "vector_history", "vector_detected_sensitive")


def _meta_to_json(meta: Dict) -> Dict:
    """A stage's output metadata as the reference writes it: the OpVectorMetadata keys
    (``vector_columns`` / ``vector_history`` / ``vector_detected_sensitive``, OpVectorMetadata.scala:187-189)
    and Spark's ``ml_attr`` attribute group at the top level, other entries (summaries) beside them."""
    out = {}
    for k, v in meta.items():
        if isinstance(v, OpVectorMetadata):
            out.update(v.to_json())
            out["ml_attr"] = {"num_attrs": len(v.columns)}
        else:
            out[k] = encode(v)
    return out


def _meta_from_json(d: Dict, name: Optional[str] = None) -> Dict:
    out = {}
    d = d or {}
    if "vector_columns" in d:
        out["vector_metadata"] = OpVectorMetadata.from_json(name or "", {k: d[k] for k in _VECTOR_KEYS if k in d})
    for k, v in d.items():
        if k in _VECTOR_KEYS or k == "ml_attr":
            continue
        if isinstance(v, dict) and "__vector_metadata__" in v:       # round-1 checkpoints
            out[k] = OpVectorMetadata.from_json(v["__vector_metadata__"], v)
        else:
            out[k] = decode(v)
    return out


def stage_to_json(st: OpPipelineStage) -> Dict:
    params = {k: encode(v) for k, v in st.params.items()}
    params["inputFeatures"] = [t.to_json() for t in st.get_transient_features()] if st._inputs else []
    params["outputFeatureName"] = st.get_output_feature_name() if (st._inputs or isinstance(
        st, FeatureGeneratorStage)) else None
    params["outputMetadata"] = _meta_to_json(st.metadata)
    return {"class": f"{type(st).__module__}.{type(st).__qualname__}", "uid": st.uid,
            "operationName": st.operation_name, "outputType": st.output_type.type_name(),
            "timestamp": int(time.time() * 1000), "paramMap": params, "defaultParamMap": {},
            "ctorArgs": encode(st.ctor_args())}


def model_to_json(model) -> Dict:
    gens = {}
    for f in list(model.raw_features) + list(model.blocklist):
        for r in (f.raw_features() if not f.is_raw else [f]):
            gens[r.origin_stage.uid] = r.origin_stage
    stages = [stage_to_json(s) for s in gens.values()] + [stage_to_json(s) for s in model.stages]
    # raw + blocklisted + every stage output (OpWorkflowModelWriter allFeatures)
    feats = {}
    for f in list(model.result_features) + list(model.blocklist):
        for x in f.traverse():
            feats[x.uid] = x
    all_features = []
    for x in feats.values():
        j = x.to_json()
        j.pop("distributions", None)
        all_features.append(j)
    rff = model.raw_feature_filter_results
    return {
        "uid": model.uid,
        "resultFeaturesUids": [f.uid for f in model.result_features],
        "blocklistedFeaturesUids": [f.uid for f in model.blocklist],
        "blocklistedMapKeys": model.blocklist_map_keys,
        "blocklistedStages": [],
        "stages": stages,
        "allFeatures": all_features,
        "parameters": model.parameters.to_string(),
        "trainParameters": model.train_parameters.to_string(),
        "rawFeatureFilterResults": json.dumps(encode(rff.to_json() if hasattr(rff, "to_json") else (rff or _EMPTY_RFF))),
        "trainTimings": encode(getattr(model, "train_timings", {})),
    }


def save_model(model, path: str, overwrite: bool = True) -> None:
    d = os.path.join(path, MODEL_DIR)
    if os.path.exists(path):
        if not overwrite:
            raise FileExistsError(path)
        if os.path.isdir(d):
            shutil.rmtree(d)
    os.makedirs(d, exist_ok=True)
    data = json.dumps(model_to_json(model), default=str).encode("utf-8")
    with gzip.open(os.path.join(d, PART + ".gz"), "wb") as f:
        f.write(data)


def _read_text(path: str) -> str:
    cands = [os.path.join(path, MODEL_DIR, PART + ".gz"), os.path.join(path, MODEL_DIR, PART),
             os.path.join(path, PART + ".gz"), os.path.join(path, PART), path]
    for c in cands:
        if os.path.isfile(c):
            if c.endswith(".gz"):
                with gzip.open(c, "rb") as f:
                    return f.read().decode("utf-8")
            with open(c) as f:
                return f.read()
    raise FileNotFoundError(f"no model found at {path}")


def _build_stage(sj: Dict) -> OpPipelineStage:
    from . import reference_compat as RC
    pm = sj.get("paramMap", {}) or {}
    is_ref = RC.is_reference_class(sj["class"])
    if is_ref and RC.simple_name(sj["class"]) != "FeatureGeneratorStage":
        st = RC.build_reference_stage(sj)
        st.uid = sj["uid"]
        st.metadata = _meta_from_json(RC.any_value(pm.get("outputMetadata")) or {}, pm.get("outputFeatureName"))
        st._output_name = pm.get("outputFeatureName")
        return st
    cls = stage_class(sj["class"])
    args = decode(RC.decode_ctor_args(sj.get("ctorArgs")) if is_ref else sj.get("ctorArgs", {}))
    if cls is FeatureGeneratorStage:
        from ..features.aggregators import aggregator_from_json, default_aggregator
        from ..stages.generator import load_extract_fn
        ef = args.get("extractFn") or {}
        tto = T.feature_type_from_name(args.get("tto", sj.get("outputType", "Text")))
        agg_j = args.get("aggregator")
        if isinstance(agg_j, dict) and is_ref:     # com.salesforce.op.aggregators.SumReal$ -> SumReal
            agg_j = {"className": RC.simple_name(agg_j.get("className", ""))}
        agg = aggregator_from_json(agg_j) or default_aggregator(tto)
        st = FeatureGeneratorStage(args.get("outputName") or pm.get("outputFeatureName"), tto,
                                   load_extract_fn(ef.get("className")), agg, args.get("aggregateWindow"),
                                   bool(args.get("outputIsResponse")), args.get("extractSource"), uid=sj["uid"],
                                   column=ef.get("column"))
        return st
    from .. import uid as _uid
    c0 = _uid.count()
    try:
        st = cls()
    except TypeError:
        st = cls.__new__(cls)
        OpPipelineStage.__init__(st, uid=sj["uid"])
    _uid.reset(c0)
    st.uid = sj["uid"]
    st.operation_name = sj.get("operationName", st.operation_name)
    if sj.get("outputType"):
        st.output_type = T.feature_type_from_name(sj["outputType"])
    for k, v in pm.items():
        if k in ("inputFeatures", "outputFeatureName", "outputMetadata"):
            continue
        st.params[k] = decode(v)
    st.metadata = _meta_from_json(pm.get("outputMetadata", {}), pm.get("outputFeatureName"))
    st._output_name = pm.get("outputFeatureName")
    st.load_ctor_args(args)
    return st


def _resolve_features(fjs: List[Dict], by_uid: Dict[str, OpPipelineStage],
                      known: Optional[Dict[str, FeatureLike]] = None) -> Dict[str, FeatureLike]:
    """Features from their JSON (``FeatureJsonHelper.fromJson``), parents first; ``known`` features (of the
    workflow) are reused by uid."""
    fmap = {f["uid"]: f for f in fjs}
    built: Dict[str, FeatureLike] = {}

    def build(uid):
        if uid in built:
            return built[uid]
        if known and uid in known and known[uid].is_raw:
            built[uid] = known[uid]
            return built[uid]
        fj = fmap[uid]
        parents = [build(p) for p in fj.get("parents", [])]
        st = by_uid.get(fj.get("originStage"))
        ftype = T.feature_type_from_name(fj["typeName"])
        if st is None and not parents and fj.get("originStage"):
            # pre-0.7 checkpoints hold no generator stages: the raw feature reads the column of its name
            from ..features.aggregators import default_aggregator
            st = FeatureGeneratorStage(fj["name"], ftype, None, default_aggregator(ftype), None,
                                       bool(fj.get("isResponse")), uid=fj["originStage"])
            by_uid[st.uid] = st
        if st is not None and not isinstance(st, FeatureGeneratorStage):
            st.output_type = ftype
        f = FeatureLike(fj["name"], ftype, fj.get("isResponse", False), st, parents, uid=fj["uid"])
        built[uid] = f
        return f

    for u in fmap:
        build(u)
    return built


def _wire(stages_j: List[Dict], by_uid: Dict[str, OpPipelineStage], built: Dict[str, FeatureLike]) -> None:
    """Set every stage's inputs (by the uids its JSON names) and output feature."""
    for sj in stages_j:
        st = by_uid[sj["uid"]]
        ins = (sj.get("paramMap", {}) or {}).get("inputFeatures", [])
        if ins:
            st._inputs = [built[t["uid"]] for t in ins]
            st._transient = [TransientFeature.from_json(t) for t in ins]
        out = next((f for f in built.values() if f.origin_stage is st), None)
        if out is not None:
            st._output = out


def load_model(path: str, workflow=None):
    """``OpWorkflowModelReader.loadJson`` (``OpWorkflowModelReader.scala:97-233``).

    Without a workflow every stage is rebuilt from the checkpoint (including ``com.salesforce.op.*``
    stages of reference-written checkpoints, :mod:`reference_compat`). With a workflow, its raw features
    (and their extract functions) replace the checkpoint's generator stages, and stages of the workflow
    with the same uid lend what a checkpoint cannot carry (user functions of lambda stages). Result
    features the checkpoint names but does not hold are dropped, as the reference does; blocklisted
    features resolve against the checkpoint's blocklisted stages and the workflow's features."""
    from ..stages.base import import_stage_modules
    from .workflow import OpWorkflowModel
    import_stage_modules()
    j = json.loads(_read_text(path))
    stages_j = j["stages"]
    wf_gens: Dict[str, OpPipelineStage] = {}
    wf_stages: Dict[str, OpPipelineStage] = {}
    wf_feats: Dict[str, FeatureLike] = {}
    if workflow is not None:
        for r in list(workflow.raw_features) + list(getattr(workflow, "blocklist", [])):
            for x in (r.raw_features() if not r.is_raw else [r]):
                wf_gens[x.origin_stage.uid] = x.origin_stage
        wf_stages = {s.uid: s for s in workflow.stages}
        for f in list(workflow.result_features) + list(getattr(workflow, "blocklist", [])):
            for x in f.traverse():
                wf_feats[x.uid] = x
    by_uid: Dict[str, OpPipelineStage] = {}
    order: List[OpPipelineStage] = []
    for sj in stages_j:
        st = wf_gens.get(sj["uid"]) or _build_stage(sj)
        orig = wf_stages.get(sj["uid"])
        if orig is not None and getattr(st, "fn", 0) is None and getattr(orig, "fn", None) is not None:
            st.fn = orig.fn
        by_uid[st.uid] = st
        order.append(st)
    built = _resolve_features(j["allFeatures"], by_uid, wf_feats)
    _wire(stages_j, by_uid, built)
    fitted = [s for s in order if not isinstance(s, FeatureGeneratorStage)]
    model = OpWorkflowModel(j.get("uid"), OpParams.from_string(j.get("parameters", "{}")))
    model.train_parameters = OpParams.from_string(j.get("trainParameters", "{}"))
    model.stages = fitted
    # OpWorkflowModelReader.resolveResultFeatures filters the loaded features by the result uids, so they come
    # back in allFeatures order (not resultFeaturesUids order)
    res_ids = set(j["resultFeaturesUids"])
    model.result_features = [built[f["uid"]] for f in j["allFeatures"] if f.get("uid") in res_ids and f["uid"] in built]
    # the raw features the result features derive from (OpWorkflowModelReader: setResultFeatures recomputes them;
    # blocklisted raw features stay in the blocklist only)
    reach = {}
    for f in model.result_features:
        for r in f.raw_features():
            reach[r.uid] = r
    if not reach:     # no result feature resolved: every raw feature of the checkpoint
        reach = {f.uid: f for f in built.values() if f.is_raw}
    model.raw_features = sorted([f for f in reach.values() if isinstance(f.origin_stage, FeatureGeneratorStage)],
                                key=lambda f: f.name)
    # blocklist (OpWorkflowModelReader.resolveBlocklist): the longer of the new / legacy field lists
    bl_feats: Dict[str, FeatureLike] = dict(wf_feats)
    for key in ("blocklistedStages", "blacklistedStages"):
        bst = j.get(key) or []
        if bst:
            extra = {}
            for sj in bst:
                st = wf_gens.get(sj["uid"]) or _build_stage(sj)
                extra[st.uid] = st
            for st in extra.values():
                if isinstance(st, FeatureGeneratorStage):     # blocklisted raw features
                    f = st.get_output()
                    bl_feats.setdefault(f.uid, f)
    bl_feats.update(built)
    lists = [j.get("blocklistedFeaturesUids") or [], j.get("blacklistedFeaturesUids") or []]
    bl = max(([bl_feats[u] for u in ids if u in bl_feats] for ids in lists), key=len)
    model.blocklist = bl
    # resolveBlocklistMapKeys: the new and the legacy field are merged with toMap -- a key present in both takes
    # the legacy field's list (the later entry wins), they are not unioned
    keys = {}
    for key in ("blocklistedMapKeys", "blacklistedMapKeys"):
        for k, v in (j.get(key) or {}).items():
            keys[k] = sorted(set(v))
    model.blocklist_map_keys = keys
    rff = j.get("rawFeatureFilterResults")
    from ..filters.raw_feature_filter import RawFeatureFilterResults
    rffj = decode(json.loads(rff)) if isinstance(rff, str) and rff else (rff or _EMPTY_RFF)
    try:
        model.raw_feature_filter_results = RawFeatureFilterResults.from_json(rffj or _EMPTY_RFF)
    except (TypeError, KeyError, ValueError):     # a shape this reader does not model: keep the JSON
        model.raw_feature_filter_results = rffj
    model.train_timings = decode(j.get("trainTimings", {}))
    if workflow is not None:
        model.reader = workflow.reader
    return model
