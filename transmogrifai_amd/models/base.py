"""Learner ABI.

The reference wraps Spark ``Predictor``s with ``OpPredictorWrapper`` (``core/.../sparkwrappers/specific/
OpPredictorWrapper.scala:71-119``) and converts fitted Spark models to ``Op*Model``s
(``SparkModelConverter.scala:64-127``) whose ``transformFn`` is ``predictRaw -> raw2probability ->
prediction`` (``OpProbabilisticClassifierModel.scala:48-76``).

Here a :class:`Learner` is a pure array-level algorithm:

* ``fit(X, y, w, params) -> state`` for one model, and
* ``fit_batch(X, y, jobs) -> [state]`` for many (params, training-rows) jobs at once -- the batched
  path the model selector uses so that every (grid point x CV fold) of a learner is trained by a
  single device program (one GEMM stream for all linear models, one level-synchronous forest for all
  trees).
* ``predict(state, X) -> (prediction, raw, probability)``.

:class:`OpPredictor` / :class:`OpPredictorModel` wrap a learner as a pipeline stage with inputs
``(label: RealNN, features: OPVector)`` and output ``Prediction``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..data.columns import PredictionColumn
from ..features import types as T
from ..stages.base import BinaryEstimator, BinaryTransformer, register_stage

_LEARNERS: Dict[str, type] = {}


def register_learner(cls):
    _LEARNERS[cls.name] = cls
    return cls


def _load_all():
    from . import glm, linear, mlp, trees  # noqa: F401  (registers every learner)


def learner_class(name: str):
    if name not in _LEARNERS:
        _load_all()
    if name not in _LEARNERS:
        raise ValueError(f"unknown learner {name}")
    return _LEARNERS[name]


@dataclass
class FitJob:
    params: Dict[str, Any]
    rows: Optional[torch.Tensor] = None       # training row ids (None = all rows)
    weights: Optional[torch.Tensor] = None    # optional per-training-row weights


def compact_rows(X: torch.Tensor, y: torch.Tensor, jobs: Sequence[FitJob]):
    """Restrict a batch of jobs to the union of their training rows.

    Cross-validation folds of a down-sampled training set touch only part of ``X``; learners that
    stream ``X`` every iteration (linear models: one pass per objective evaluation) then read the
    union once instead of all ``N`` rows per pass. Returns ``(X_u, y_u, jobs_u)`` with row ids
    remapped, or the inputs unchanged when a job uses every row or the union is all of ``X``."""
    if not jobs or any(j.rows is None for j in jobs):
        return X, y, list(jobs)
    # jobs that share a row set (the grid points of one fold) keep sharing one remapped tensor, so the learners
    # can still group them by it (one weight column / statistic per fold, models/linear.py)
    keys, uniq, which = {}, [], []
    for j in jobs:
        k = (j.rows.data_ptr(), int(j.rows.numel()), tuple(j.rows.stride()), j.rows.device)
        if k not in keys:
            keys[k] = len(uniq)
            uniq.append(j.rows)
        which.append(keys[k])
    U, parts = union_rows(uniq, X.shape[0], X.device)
    if U.numel() >= X.shape[0]:
        return X, y, list(jobs)
    return X.index_select(0, U), y.to(X.device).index_select(0, U), \
        [FitJob(j.params, parts[i], j.weights) for j, i in zip(jobs, which)]


def union_rows(rows: Sequence[torch.Tensor], N: int, device):
    """Sorted union ``U`` of several row-id sets over ``[0, N)`` and each set remapped to positions in
    ``U``: a presence mask + prefix count (O(N), no sort; ``torch.unique`` sorts the concatenation)."""
    cat = torch.cat([r.to(device) for r in rows]).to(torch.int64)
    mask = torch.zeros(N, dtype=torch.bool, device=device)
    mask[cat] = True
    U = mask.nonzero().squeeze(1)
    pos = torch.cumsum(mask, 0) - 1
    parts = torch.split(pos[cat], [int(r.numel()) for r in rows])
    return U, list(parts)


class Learner:
    name = "Learner"
    problem = "binary"          # binary | multiclass | regression
    defaults: Dict[str, Any] = {}
    # intra-job parallelism over ranks (parallel/learner_parallel.py): "rows" (linear models),
    # "features" (boosted / single trees) or None (jobs sharded whole over the ranks)
    parallel: Optional[str] = None

    def __init__(self, **params):
        p = dict(self.defaults)
        p.update(params)
        self.params = p

    # -- single model -------------------------------------------------------------------------
    def fit(self, X: torch.Tensor, y: torch.Tensor, w: Optional[torch.Tensor] = None,
            params: Optional[dict] = None, context=None) -> dict:
        p = dict(self.params)
        p.update(params or {})
        return self.fit_batch(X, y, [FitJob(p, None, w)], context=context)[0]

    # -- many models --------------------------------------------------------------------------
    def fit_batch(self, X: torch.Tensor, y: torch.Tensor, jobs: Sequence[FitJob], context=None) -> List[dict]:
        raise NotImplementedError

    def predict(self, state: dict, X: torch.Tensor, context=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        raise NotImplementedError

    def predict_batch(self, states: Sequence[dict], X: torch.Tensor, rows: Sequence[Optional[torch.Tensor]],
                      context=None):
        """Predictions of many models on row subsets (default: one call per model)."""
        out = []
        for s, r in zip(states, rows):
            Xr = X if r is None else X[r]
            out.append(self.predict(s, Xr, context))
        return out

    def n_classes(self, state) -> int:
        return int(state.get("n_classes", 2))

    def feature_contributions(self, state, d: int) -> Optional[np.ndarray]:
        return None

    def state_to_json(self, state: dict) -> dict:
        from ..utils.serde import encode
        return encode(state)

    def state_from_json(self, d: dict) -> dict:
        from ..utils.serde import decode
        return decode(d)

    def summary(self, params) -> Dict[str, Any]:
        return dict(params)


def probability_outputs(raw: torch.Tensor, binary_margin: bool = True, threshold: float = 0.5):
    """(prediction, raw, probability) from a logistic margin ``[N]``."""
    m = raw.to(torch.float64)
    p1 = torch.sigmoid(m)
    rawp = torch.stack([-m, m], 1)
    prob = torch.stack([1 - p1, p1], 1)
    pred = (p1 > threshold).to(torch.float64)
    return pred, rawp, prob


# ------------------------------------------------------------------------------------------ stages
PREDICT_CHUNK_ROWS = 2_000_000


def predict_chunked(learner, state, vec, chunk: int = PREDICT_CHUNK_ROWS):
    """``learner.predict`` over a (possibly blocked) vector column in row chunks, so scoring never
    materialises the whole feature matrix (the blocked view is gathered ``chunk`` rows at a time)."""
    n = len(vec)
    if not getattr(vec, "is_blocked", False) and n <= chunk:
        return learner.predict(state, vec.values)
    outs = []
    for a in range(0, max(n, 1), chunk):
        b = min(n, a + chunk)
        rows = torch.arange(a, b, device=vec.device)
        outs.append(learner.predict(state, vec.take_rows(rows)))
    if len(outs) == 1:
        return outs[0]
    return tuple(torch.cat([o[i] for o in outs], 0) for i in range(3))


@register_stage
class OpPredictorModel(BinaryTransformer):
    """A fitted learner as a pipeline stage (label, features) -> Prediction."""
    output_type = T.Prediction
    allow_label_as_input = True

    def __init__(self, learner_name: str = "", state: Optional[dict] = None, params: Optional[dict] = None,
                 uid=None, **kw):
        super().__init__(None, uid=uid, **kw)
        self.learner_name = learner_name
        self.state = state
        self.learner_params = dict(params or {})

    @property
    def learner(self) -> Learner:
        return learner_class(self.learner_name)(**self.learner_params)

    def transform_columns(self, *cols, ds=None):
        pred, raw, prob = predict_chunked(self.learner, self.state, cols[1])
        return PredictionColumn(pred.to(torch.float64), raw.to(torch.float64), prob.to(torch.float64))

    def transform_row(self, *values):
        x = torch.as_tensor(np.asarray(values[1], np.float64))[None, :]
        pred, raw, prob = self.learner.predict(self.state, x)
        return T.Prediction(prediction=float(pred[0]), raw_prediction=raw[0].tolist(),
                            probability=prob[0].tolist()).value

    def ctor_args(self):
        return {"learner": self.learner_name, "params": _jsonable(self.learner_params),
                "state": self.learner.state_to_json(self.state)}

    def load_ctor_args(self, a):
        self.learner_name = a["learner"]
        self.learner_params = dict(a.get("params", {}))
        self.state = self.learner.state_from_json(a["state"])


class OpPredictor(BinaryEstimator):
    """Estimator stage wrapping one learner with fixed params."""
    output_type = T.Prediction
    allow_label_as_input = True
    learner_cls: type = Learner

    def __init__(self, uid=None, **params):
        super().__init__(uid=uid)
        self.params.update(self.learner_cls.defaults)
        self.params.update(params)

    def _accepts_param(self, name):
        return name in self.learner_cls.defaults

    def fit_columns(self, label_col, vec_col, ds=None):
        X = vec_col.values
        y = label_col.values.to(X.dtype)
        learner = self.learner_cls(**self.params)
        state = learner.fit(X, y)
        return OpPredictorModel(self.learner_cls.name, state, dict(self.params))


def _jsonable(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, (np.floating, np.integer)):
            v = v.item()
        out[k] = v
    return out
