"""Spark-free scoring of a fitted workflow model (``local/.../OpWorkflowModelLocal.scala:79-122``).

Two serving paths:

* :func:`score_function` -- single-record, low-latency CPU row path. Returns ``f(record) -> dict`` that
  folds the record through every fitted stage with ``transform_key_value`` (the reference's
  ``scoreFunction``); raw features are extracted from the record by each generator stage.
* :func:`batch_score_function` -- micro-batch path: records are turned into columnar datasets on the
  engine device and pushed through the fused columnar transforms (the same kernels as training),
  which is the throughput path on a GPU.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Iterable, List, Optional

from ..data.dataset import Dataset
from ..stages.base import OpTransformer


def _ordered_stages(model) -> List[OpTransformer]:
    from ..workflow.dag import compute_dag
    by_uid = {s.uid: s for s in model.stages}
    out = []
    for layer in compute_dag(model.result_features):
        for st, _ in layer:
            fs = by_uid.get(st.uid)
            if fs is not None:
                out.append(fs)
    return out


def score_function(model) -> Callable[[Dict[str, Any]], Dict[str, Any]]:
    """``record -> {result feature name: value}``; record keys are raw feature (or source column) names."""
    stages = _ordered_stages(model)
    raws = list(model.raw_features)
    result_names = [f.name for f in model.result_features]

    def fn(record: Dict[str, Any]) -> Dict[str, Any]:
        row: Dict[str, Any] = {}
        for f in raws:
            st = f.origin_stage
            v = st.extract(record) if st is not None and hasattr(st, "extract") else record.get(f.name)
            row[f.name] = v.value if hasattr(v, "value") and not isinstance(v, (dict, list)) else v
        for st in stages:
            row[st.get_output_feature_name()] = st.transform_key_value(row.get)
        return {n: row.get(n) for n in result_names}

    return fn


def batch_score_function(model, device=None) -> Callable[[Iterable[Dict[str, Any]]], List[Dict[str, Any]]]:
    """``records -> [result dict]`` through the columnar (device) transforms."""
    from ..config import default_device
    from ..readers.base import dataset_from_records

    dev = device or default_device()

    def fn(records) -> List[Dict[str, Any]]:
        recs = list(records)
        ds: Dataset = dataset_from_records(recs, model.raw_features, dev)
        out = model.transform_dataset(ds)
        names = [f.name for f in model.result_features]
        return out.to_rows(names)

    return fn
