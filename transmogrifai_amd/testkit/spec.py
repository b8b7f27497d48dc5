"""Reusable stage contract checks (``OpTransformerSpec.scala:59-89``, ``TransformerSpecCommon`` ``:122-177``,
``OpEstimatorSpec.scala:82-142``): every stage must agree across

* the batch (columnar / device) path ``stage.transform(dataset)``,
* the per-row path ``stage.transform_row(*values)`` (local scoring),
* the key/value path ``transform_key_value(getter)``,
* a JSON write -> read round trip of the (fitted) stage, and
* empty input (zero rows).
"""
from __future__ import annotations

import json
import math
from typing import Optional

import numpy as np
import torch

from ..data.dataset import Dataset
from ..stages.base import OpEstimator, OpTransformer


def _norm(v):
    if isinstance(v, torch.Tensor):
        v = v.detach().cpu().numpy()
    if isinstance(v, np.ndarray):
        return [float(x) for x in v.reshape(-1)]
    if isinstance(v, (frozenset, set)):
        return sorted(v)
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in sorted(v.items())}
    if isinstance(v, (list, tuple)):
        return [_norm(x) for x in v]
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (np.integer,)):
        return int(v)
    return v


def values_close(a, b, tol: float = 1e-6) -> bool:
    a, b = _norm(a), _norm(b)
    if isinstance(a, float) and isinstance(b, (int, float)) or isinstance(b, float) and isinstance(a, (int, float)):
        if math.isnan(float(a)) and math.isnan(float(b)):
            return True
        return abs(float(a) - float(b)) <= tol * max(1.0, abs(float(a)), abs(float(b)))
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(values_close(x, y, tol) for x, y in zip(a, b))
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(values_close(a[k], b[k], tol) for k in a)
    return a == b


def roundtrip(stage: OpTransformer) -> OpTransformer:
    """Serialize a stage to the checkpoint JSON form and rebuild it (inputs re-wired)."""
    from ..workflow.io import _build_stage, stage_to_json
    js = json.loads(json.dumps(stage_to_json(stage), default=str))
    st = _build_stage(js)
    st._inputs = list(stage._inputs)
    st._transient = stage._transient
    st._output = stage._output
    st._output_name = stage._output_name
    return st


def check_transformer(stage: OpTransformer, ds: Dataset, expected=None, tol: float = 1e-6,
                      check_rows: bool = True, check_roundtrip: bool = True) -> list:
    """Run the contract checks; returns the batch output values (python list)."""
    out = stage.transform(ds)
    name = stage.get_output().name
    assert name in out, f"output column {name} missing"
    batch = out[name].to_list()
    assert len(batch) == len(ds)
    if expected is not None:
        assert len(expected) == len(batch)
        for i, (g, e) in enumerate(zip(batch, expected)):
            assert values_close(g, e, tol), f"row {i}: got {g!r} expected {e!r}"
    inputs = [f.name for f in stage.get_input_features()]
    if check_rows:
        for i in range(len(ds)):
            vals = [ds[n].row(i) for n in inputs]
            r = stage.transform_row(*vals)
            assert values_close(r, batch[i], tol), f"row path differs at {i}: {r!r} vs {batch[i]!r}"
            row = {n: ds[n].row(i) for n in inputs}
            kv = stage.transform_key_value(row.get)
            assert values_close(kv, batch[i], tol), f"key/value path differs at {i}"
    if check_roundtrip:
        st2 = roundtrip(stage)
        again = st2.transform(ds)[name].to_list()
        for i, (a, b) in enumerate(zip(again, batch)):
            assert values_close(a, b, tol), f"reloaded stage differs at {i}: {a!r} vs {b!r}"
    empty = ds.take(torch.zeros(0, dtype=torch.long))
    e_out = stage.transform(empty)
    assert len(e_out[name]) == 0
    return [_norm(v) for v in batch]


def check_estimator(est: OpEstimator, ds: Dataset, expected=None, tol: float = 1e-6, **kw):
    model = est.fit(ds)
    assert model.uid == est.uid
    assert model.parent is est
    batch = check_transformer(model, ds, expected, tol, **kw)
    return model, batch
