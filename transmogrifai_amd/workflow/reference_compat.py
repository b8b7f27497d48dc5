"""Reading checkpoints written by the reference (``com.salesforce.op.*`` stage classes).

The reference stage writer stores Spark ``paramMap`` entries under camelCase names and the constructor
arguments of a stage as ``AnyValue`` records (``DefaultOpPipelineStageReaderWriter.scala:58-176``:
``{"type": "Value" | "TypeTag" | "ClassInstance" | "SparkWrappedStage", "value": ...}``). This module
maps the stages the reference's own fixtures hold (``core/src/test/resources/OldModelVersion*``) onto
this package's stage classes:

* transformers whose state is only params: ``RealNNVectorizer``, ``BinaryVectorizer``,
  ``DateListVectorizer`` (``withTimeSince`` / ``first`` / ``fillWithPivotMode*`` -> one ``pivot``);
* fitted vectorizer models whose state is in ``ctorArgs``: ``RealVectorizerModel`` /
  ``IntegralVectorizerModel`` (``fillValues``), ``OpSetVectorizerModel`` / ``OpTextPivotVectorizerModel``
  (``topValues``), ``SmartTextVectorizerModel`` (``args``: ``isCategorical`` or ``vectorizationMethods``,
  ``topValues``, ``hashingParams``), ``VectorsCombinerModel``;
* ``UnaryLambdaTransformer`` and the other lambda stages: the function class name resolves through the
  function registry (``stages/generator.py``) -- loading never imports or reflects user code.

A stage class that is not mapped raises with the list of supported classes: a checkpoint is never
half-loaded silently.
"""
from __future__ import annotations

import re
from typing import Any, Callable, Dict

from ..features import types as T

REFERENCE_PREFIX = "com.salesforce.op."


def is_reference_class(name: str) -> bool:
    return isinstance(name, str) and name.startswith(REFERENCE_PREFIX)


def simple_name(name: str) -> str:
    return name.rsplit(".", 1)[-1].rstrip("$")


def any_value(v: Any) -> Any:
    """Unwrap one ``AnyValue`` record (plain JSON passes through)."""
    if isinstance(v, dict) and v.get("type") in ("Value", "TypeTag", "ClassInstance", "SparkWrappedStage") \
            and "value" in v:
        if v["type"] == "ClassInstance":
            return {"className": v["value"]}
        if v["type"] == "SparkWrappedStage":
            raise ValueError("checkpoint holds a Spark-wrapped (MLeap) stage; only native stages can be read")
        return v["value"]
    return v


def decode_ctor_args(args: Dict[str, Any]) -> Dict[str, Any]:
    return {k: any_value(v) for k, v in (args or {}).items()}


def snake(k: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", k).lower()


def _set_known(st, pm: Dict[str, Any], skip=()) -> None:
    """Copy reference params whose snake_case name the stage accepts."""
    for k, v in pm.items():
        if k in skip or k in ("inputFeatures", "outputFeatureName", "outputMetadata", "inputSchema"):
            continue
        name = snake(k)
        if name in st.params or st._accepts_param(name):
            st.params[name] = v


# --------------------------------------------------------------------------------------- adapters
def _real_nn(pm, a):
    from ..stages.feature.vectorizers import RealNNVectorizer
    return RealNNVectorizer()


def _binary(pm, a):
    from ..stages.feature.vectorizers import BinaryVectorizer
    st = BinaryVectorizer()
    _set_known(st, pm)
    return st


def _date_list(pm, a):
    """``DateListVectorizer.scala:60-120``: withTimeSince (+ first) or one of the mode pivots."""
    from ..stages.feature.vectorizers import DateListVectorizer
    st = DateListVectorizer()
    if pm.get("fillWithPivotModeDay"):
        pv = "ModeDay"
    elif pm.get("fillWithPivotModeMonth"):
        pv = "ModeMonth"
    elif pm.get("fillWithPivotModeHour"):
        pv = "ModeHour"
    else:
        pv = "SinceFirst" if pm.get("first", True) else "SinceLast"
    st.params["pivot"] = pv
    if pm.get("referenceDate") is not None:
        st.params["reference_date"] = int(pm["referenceDate"])
    st.params["track_nulls"] = bool(pm.get("trackNulls", True))
    st.params["fill_value"] = float(pm.get("fillValue", 0.0))
    return st


def _real_model(op_name):
    def build(pm, a):
        from ..stages.feature.vectorizers import RealVectorizerModel
        st = RealVectorizerModel([float(x) for x in a.get("fillValues", [])], bool(a.get("trackNulls", True)))
        st.operation_name = a.get("operationName", op_name)
        return st
    return build


def _pivot_model(pm, a):
    from ..stages.feature.vectorizers import OpOneHotVectorizerModel
    st = OpOneHotVectorizerModel(a.get("topValues") or [], bool(a.get("shouldCleanText", True)),
                                 bool(a.get("shouldTrackNulls", True)))
    st.operation_name = a.get("operationName", "vecSet")
    return st


def _hashing(h: Dict[str, Any]):
    from ..stages.feature.vectorizers import HashingParams
    h = h or {}
    return HashingParams(num_features=int(h.get("numFeatures", 512)), num_inputs=int(h.get("numInputs", 1)),
                         max_num_features=int(h.get("maxNumOfFeatures", 1 << 17)),
                         binary=bool(h.get("binaryFreq", False)),
                         prepend_feature_name=bool(h.get("prependFeatureName", True)),
                         hash_space_strategy=str(h.get("hashSpaceStrategy", "Auto")).lower(),
                         hash_with_index=bool(h.get("hashWithIndex", False)))


def _smart_text_model(pm, a):
    """``SmartTextVectorizerModel(args: SmartTextVectorizerModelArgs)``: older checkpoints carry
    ``isCategorical`` (pivot vs hash), newer ones ``vectorizationMethods``."""
    from ..stages.feature.vectorizers import SmartTextVectorizerModel
    args = a.get("args", a)
    if "vectorizationMethods" in args:
        methods = [str(m).lower() for m in args["vectorizationMethods"]]
    else:
        methods = ["pivot" if c else "hash" for c in args.get("isCategorical", [])]
    st = SmartTextVectorizerModel(methods, args.get("topValues") or [[] for _ in methods],
                                  bool(args.get("shouldCleanText", True)), bool(args.get("shouldTrackNulls", True)),
                                  _hashing(args.get("hashingParams")),
                                  bool(args.get("shouldTrackLen", args.get("trackTextLen", False))),
                                  int(pm.get("minTokenLength", 1)), bool(pm.get("toLowercase", True)))
    st.operation_name = a.get("operationName", "smartTxtVec")
    return st


def _combiner_model(pm, a):
    from ..stages.feature.vectorizers import VectorsCombinerModel
    return VectorsCombinerModel()


def _lambda(pm, a):
    """``UnaryLambdaTransformer(operationName, transformFn)`` (``UnaryTransformer.scala:128``): the
    function is selected from the registry by its class name."""
    from ..stages.feature.misc_stages import MapTransformer
    from ..stages.generator import load_extract_fn
    fn_ref = a.get("transformFn") or {}
    name = fn_ref.get("className") if isinstance(fn_ref, dict) else fn_ref
    st = MapTransformer(None, None, a.get("operationName"))
    st.fn = load_extract_fn(name) if name else None
    return st


def _index_to_string(no_filter: bool):
    """``OpIndexToString`` (a Spark ``IndexToString`` wrapper, ``OpIndexToString.scala:50-74``) and
    ``OpIndexToStringNoFilter(labels, unseenName)``: the labels come from the wrapped stage's params (or the
    ctor args); empty labels fall back to the input indexer's metadata at transform time."""
    def build(pm, a):
        from ..stages.feature.indexers import OpIndexToString, OpIndexToStringNoFilter
        spark = pm.get("sparkMlStage") if isinstance(pm.get("sparkMlStage"), dict) else {}
        labels = list(a.get("labels") or pm.get("labels") or spark.get("labels") or [])
        if no_filter:
            return OpIndexToStringNoFilter(labels=labels, unseen_name=str(a.get("unseenName", "UnseenIndex")))
        return OpIndexToString(labels=labels)
    return build


ADAPTERS: Dict[str, Callable] = {
    "OpIndexToString": _index_to_string(False),
    "OpIndexToStringNoFilter": _index_to_string(True),
    "RealNNVectorizer": _real_nn,
    "BinaryVectorizer": _binary,
    "DateListVectorizer": _date_list,
    "RealVectorizerModel": _real_model("vecReal"),
    "IntegralVectorizerModel": _real_model("vecInt"),
    "OpSetVectorizerModel": _pivot_model,
    "OpTextPivotVectorizerModel": _pivot_model,
    "SmartTextVectorizerModel": _smart_text_model,
    "VectorsCombinerModel": _combiner_model,
    "UnaryLambdaTransformer": _lambda,
}


def build_reference_stage(sj: Dict[str, Any]):
    """One reference stage JSON -> a stage of this package (uid, output type, output metadata set by
    the caller)."""
    name = simple_name(sj["class"])
    ad = ADAPTERS.get(name)
    if ad is None:
        raise ValueError(f"reference stage class {sj['class']!r} is not supported by this reader "
                         f"(supported: FeatureGeneratorStage, {', '.join(sorted(ADAPTERS))})")
    pm = {k: any_value(v) for k, v in (sj.get("paramMap") or {}).items()}
    a = decode_ctor_args(sj.get("ctorArgs"))
    st = ad(pm, a)
    tto = a.get("tto")
    if tto and isinstance(tto, str):
        try:
            st.output_type = T.feature_type_from_name(tto)
        except ValueError:
            pass
    return st
