"""DAG computation and layer-by-layer fit / transform.

Reference: ``FitStagesUtil`` (``core/.../utils/stages/FitStagesUtil.scala:51-369``): ``computeDAG`` (stages layered by
distance, deepest first, each stage once, ``:173-198``), ``fitAndTransformDAG`` / ``fitAndTransformLayer``
(``:212-290``: fit the estimators of a layer on train, evaluate ``HasTestEval`` models on the hold-out,
then apply every transformer of the layer to train and test) and ``cutDAG`` (``:302-355``) for
workflow-level CV. A layer's transformers write new device columns into the columnar dataset -- no
row materialization.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

from ..data.dataset import Dataset
from ..stages.base import OpEstimator, OpTransformer

log = logging.getLogger(__name__)

Layer = List[Tuple[object, int]]

_MEM_TRACE = os.environ.get("TMOG_MEM_TRACE") == "1"
_STAGE_SYNC = os.environ.get("TMOG_STAGE_SYNC") == "1"


def _clock() -> float:
    """Stage timer; ``TMOG_STAGE_SYNC=1`` drains the device first so asynchronous kernels are charged to the
    stage that launched them (profiling only: it serialises the host with the GPU)."""
    if _STAGE_SYNC:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    return time.time()


def compute_dag(features) -> List[Layer]:
    by_dist: Dict[int, list] = {}
    for f in features:
        for st, d in f.parent_stages().items():
            by_dist.setdefault(d, []).append((st, d))
    layers = []
    seen = set()
    for d in sorted(by_dist, reverse=True):
        layer = []
        for st, dd in sorted(by_dist[d], key=lambda sd: sd[0].get_output_feature_name()):
            if id(st) in seen:
                continue
            seen.add(id(st))
            layer.append((st, dd))
        if layer:
            layers.append(layer)
    return layers


def fit_and_transform_layer(layer: Layer, train: Dataset, test: Optional[Dataset], timings: Optional[dict] = None):
    fitted = []
    for st, _ in layer:
        t0 = _clock()
        if isinstance(st, OpEstimator):
            m = st.fit(train)
            if test is not None and len(test) > 0 and hasattr(m, "evaluate_model"):
                test_in = test
                m.evaluate_model(test_in)
            fitted.append(m)
        else:
            fitted.append(st)
        if timings is not None:
            timings[f"fit:{st.stage_name()}"] = _clock() - t0
    for m in fitted:
        t0 = _clock()
        train = m.transform(train)
        if test is not None and len(test) > 0:
            test = m.transform(test)
        if timings is not None:
            timings[f"transform:{m.stage_name()}"] = _clock() - t0
        _mem_mark(timings, f"transform:{m.stage_name()}")
    return train, test, fitted


def fit_and_transform_dag(dag: Sequence[Layer], train, test: Optional[Dataset] = None,
                          timings: Optional[dict] = None, keep: Optional[set] = None):
    """Fit and apply the DAG layer by layer.

    With ``keep`` given (the column names some later DAG part still reads), a column is dropped from
    ``train`` / ``test`` right after the transform of its last consumer inside this DAG, so raw columns
    and intermediate vector blocks do not outlive their use (the feature matrix of a 10M-row table is
    tens of GB; only the final selector's input has to stay resident)."""
    if isinstance(train, list):      # handed over as [train, test]: emptied here, so the caller keeps no
        box = train                  # reference and columns dropped below are really released
        train, test = box[0], box[1]
        box.clear()
    last = _last_uses(dag) if keep is not None else {}
    fitted_all = []
    for li, layer in enumerate(dag):
        # a hold-out must be transformed before a HasTestEval model of the next layer evaluates on it
        train, test, fitted = _fit_layer_with_eval(layer, train, test, timings, li, last, keep)
        fitted_all.extend(fitted)
    return train, test, fitted_all


def _last_uses(dag: Sequence[Layer]) -> Dict[str, Tuple[int, int]]:
    last: Dict[str, Tuple[int, int]] = {}
    for li, layer in enumerate(dag):
        for si, (st, _) in enumerate(layer):
            for f in st.get_input_features():
                last[f.name] = max(last.get(f.name, (li, si)), (li, si))
    return last


def _mem_mark(timings, what):
    """``TMOG_MEM_TRACE=1``: record the device memory high-water mark of each stage fit / transform."""
    if timings is None or not _MEM_TRACE:
        return
    import torch
    if torch.cuda.is_available():
        timings[f"peak_gb:{what}"] = round(torch.cuda.max_memory_allocated() / 1e9, 3)
        torch.cuda.reset_peak_memory_stats()


def _fit_layer_with_eval(layer, train, test, timings, li=0, last=None, keep=None):
    from ..utils import listener as L
    fitted = []
    for st, _ in layer:
        t0 = _clock()
        if isinstance(st, OpEstimator):
            with L.stage(st.stage_name(), "fit", len(train)):
                m = st.fit(train)
                if test is not None and len(test) > 0 and hasattr(m, "evaluate_model"):
                    m.evaluate_model(test)
            fitted.append(m)
        else:
            fitted.append(st)
        if timings is not None:
            timings[f"fit:{st.stage_name()}"] = _clock() - t0
        _mem_mark(timings, f"fit:{st.stage_name()}")
    for si, m in enumerate(fitted):
        t0 = _clock()
        with L.stage(m.stage_name(), "transform", len(train) + (len(test) if test is not None else 0)):
            train = m.transform(train)
            if test is not None and len(test) > 0:
                test = m.transform(test)
        if keep is not None and last:
            dead = [n for n, pos in last.items() if pos == (li, si) and n not in keep]
            if dead:
                train = train.drop(dead)
                if test is not None:
                    test = test.drop(dead)
        if timings is not None:
            timings[f"transform:{m.stage_name()}"] = _clock() - t0
        _mem_mark(timings, f"transform:{m.stage_name()}")
    return train, test, fitted


def apply_transformations_dag(data: Dataset, dag: Sequence[Layer]) -> Dataset:
    """Score path: apply already-fitted transformers layer by layer (``OpWorkflowCore.scala:324-348``)."""
    for layer in dag:
        for st, _ in layer:
            if isinstance(st, OpEstimator):
                raise ValueError(f"stage {st.uid} is not fitted")
            data = st.transform(data)
    return data


def cut_dag(dag: Sequence[Layer]):
    """Split a DAG around its model selector for workflow-level CV (``FitStagesUtil.cutDAG``)."""
    from ..selector.model_selector import ModelSelector
    sels = [(st, d) for layer in dag for st, d in layer if isinstance(st, ModelSelector)]
    if not sels:        # nothing to cut (OpWorkflowCore.cutDAG: CutDAG(None, empty, empty, empty))
        return None, [], [], []
    if len(sels) > 1:
        raise ValueError(f"OpWorkflow can contain at most 1 Model Selector. Found {len(sels)}")
    ms, dist = sels[0]
    after = [layer for layer in dag if any(d < dist for _, d in layer)]
    before = [layer for layer in dag if not any(d < dist for _, d in layer)]
    ms_dag = compute_dag([ms.get_output()])[:-1]
    ms_dag = [[(st, d + len(after)) for st, d in layer] for layer in ms_dag]
    non_ms = [[(st, d) for st, d in layer if st is not ms] for layer in before]
    non_ms = [l for l in non_ms if l]
    first = next((i for i, layer in enumerate(ms_dag)
                  if any(any(t.is_response for t in st.get_input_features()) and
                         any(not t.is_response for t in st.get_input_features()) for st, _ in layer)), -1)
    if first == -1:
        return ms, non_ms, [], after
    during = ms_dag[first:]
    flat = {id(st) for layer in during for st, _ in layer}
    before2 = [[(st, d) for st, d in layer if id(st) not in flat] for layer in non_ms]
    return ms, [l for l in before2 if l], during, after


def copy_dag(dag: Sequence[Layer]) -> List[Layer]:
    """Fresh stage copies of a DAG (``stage.copy(ParamMap.empty)`` per fold in OpCrossValidation.scala:
    107-112): same uid, inputs and params, private params / metadata, so fitting a copy never
    touches the workflow's own stages."""
    import copy
    out = []
    for layer in dag:
        nl = []
        for st, d in layer:
            c = copy.copy(st)
            c.params = dict(getattr(st, "params", {}))
            c.metadata = copy.deepcopy(getattr(st, "metadata", {}))
            nl.append((c, d))
        out.append(nl)
    return out
