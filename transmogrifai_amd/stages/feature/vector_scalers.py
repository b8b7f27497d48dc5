"""Vector-level Spark-ML feature estimators the reference reaches through ``OpEstimatorWrapper`` /
``OpTransformerWrapper`` (``features/.../sparkwrappers/generic/SwUnaryEstimator.scala``; exercised on
``StandardScaler`` in ``OpWorkflowModelReaderWriterTest.scala:144-159``): standard, min-max and max-abs scaling,
p-norm normalisation and PCA over an ``OPVector``, with Spark's semantics.

Every statistic is one column reduction over the device-resident ``[n, d]`` matrix (fp64 accumulation); PCA is
one Gram GEMM plus a ``d x d`` symmetric eigen-decomposition; transforms are fused elementwise / GEMM ops on the
device. Scalers keep the input's vector metadata (the columns keep their meaning), PCA names its outputs
``<input>_pca_<i>``.
"""
from __future__ import annotations

from typing import Optional

import torch

from ...data.columns import VectorColumn
from ...data.vector_metadata import OpVectorColumnMetadata, OpVectorMetadata
from ...features import types as T
from ..base import OpTransformer, UnaryEstimator, register_stage


def _same_meta(stage, v: VectorColumn) -> Optional[OpVectorMetadata]:
    m = v.metadata
    if m is None:
        return None
    return m.select(list(range(len(m.columns))), stage.get_output_feature_name())


def _f64(v: VectorColumn) -> torch.Tensor:
    return v.values.to(torch.float64)


class _VectorModel(OpTransformer):
    output_type = T.OPVector
    arity = 1
    _state = ()

    def __init__(self, uid=None, **kw):
        super().__init__(uid=uid, **kw)
        for k in self._state:
            setattr(self, k, None)

    def ctor_args(self):
        return {k: (getattr(self, k).cpu().tolist() if isinstance(getattr(self, k), torch.Tensor)
                    else getattr(self, k)) for k in self._state}

    def load_ctor_args(self, a):
        for k in self._state:
            v = a.get(k)
            setattr(self, k, torch.tensor(v, dtype=torch.float64) if isinstance(v, list) else v)

    def _t(self, name, dev):
        t = getattr(self, name)
        if t.device != dev:
            t = t.to(dev)
            setattr(self, name, t)
        return t

    def _out(self, v: VectorColumn, x: torch.Tensor) -> VectorColumn:
        meta = self.metadata.get("vector_metadata") or _same_meta(self, v)
        if meta is not None:
            self.metadata["vector_metadata"] = meta
        return VectorColumn(x.to(v.values.dtype), meta)


@register_stage
class OpStandardScalerModel(_VectorModel):
    operation_name = "stdScaled"
    _state = ("mean", "std")

    def transform_columns(self, v, ds=None):
        x = _f64(v)
        dev = x.device
        if self.params.get("with_mean"):
            x = x - self._t("mean", dev)
        if self.params.get("with_std", True):
            s = self._t("std", dev)
            x = torch.where(s > 0, x / torch.where(s > 0, s, torch.ones_like(s)), torch.zeros_like(x))
        return self._out(v, x)


@register_stage
class OpStandardScaler(UnaryEstimator):
    """Spark ``StandardScaler``: unit (sample, n - 1) standard deviation, optional centring; a zero-variance column
    scales to 0."""
    operation_name = "stdScaled"
    output_type = T.OPVector
    _defaults = {"with_mean": False, "with_std": True}

    def fit_columns(self, v, ds=None):
        x = _f64(v)
        n = x.shape[0]
        m = OpStandardScalerModel()
        m.mean = x.mean(0) if n else torch.zeros(x.shape[1], dtype=torch.float64, device=x.device)
        m.std = x.std(0, unbiased=True) if n > 1 else torch.zeros_like(m.mean)
        m.params.update(self.params)
        return m


@register_stage
class OpMinMaxScalerModel(_VectorModel):
    operation_name = "minMaxScaled"
    _state = ("lo", "hi")

    def transform_columns(self, v, ds=None):
        x = _f64(v)
        dev = x.device
        lo, hi = self._t("lo", dev), self._t("hi", dev)
        a, b = float(self.params.get("min", 0.0)), float(self.params.get("max", 1.0))
        rng = hi - lo
        scaled = (x - lo) / torch.where(rng != 0, rng, torch.ones_like(rng)) * (b - a) + a
        return self._out(v, torch.where(rng != 0, scaled, torch.full_like(x, 0.5 * (a + b))))


@register_stage
class OpMinMaxScaler(UnaryEstimator):
    """Spark ``MinMaxScaler``: each column rescaled to ``[min, max]``; a constant column maps to the middle."""
    operation_name = "minMaxScaled"
    output_type = T.OPVector
    _defaults = {"min": 0.0, "max": 1.0}

    def fit_columns(self, v, ds=None):
        x = _f64(v)
        m = OpMinMaxScalerModel()
        m.lo, m.hi = (x.min(0).values, x.max(0).values) if x.shape[0] else \
            (torch.zeros(x.shape[1], dtype=torch.float64, device=x.device),) * 2
        m.params.update(self.params)
        return m


@register_stage
class OpMaxAbsScalerModel(_VectorModel):
    operation_name = "maxAbsScaled"
    _state = ("max_abs",)

    def transform_columns(self, v, ds=None):
        x = _f64(v)
        s = self._t("max_abs", x.device)
        return self._out(v, x / torch.where(s > 0, s, torch.ones_like(s)))


@register_stage
class OpMaxAbsScaler(UnaryEstimator):
    """Spark ``MaxAbsScaler``: each column divided by its largest absolute value (all-zero columns unchanged)."""
    operation_name = "maxAbsScaled"
    output_type = T.OPVector

    def fit_columns(self, v, ds=None):
        x = _f64(v)
        m = OpMaxAbsScalerModel()
        m.max_abs = x.abs().max(0).values if x.shape[0] else torch.zeros(x.shape[1], dtype=torch.float64,
                                                                         device=x.device)
        return m


@register_stage
class OpNormalizer(_VectorModel):
    """Spark ``Normalizer``: every row divided by its p-norm (``p = inf``: the max-abs norm); zero rows stay zero."""
    operation_name = "normalized"
    _defaults = {"p": 2.0}

    def transform_columns(self, v, ds=None):
        x = _f64(v)
        p = float(self.params.get("p", 2.0))
        nrm = torch.linalg.vector_norm(x, ord=p, dim=1, keepdim=True)
        return self._out(v, x / torch.where(nrm > 0, nrm, torch.ones_like(nrm)))


@register_stage
class OpPCAModel(_VectorModel):
    operation_name = "pca"
    _state = ("pc", "explained_variance")

    def transform_columns(self, v, ds=None):
        x = _f64(v)
        pc = self._t("pc", x.device)
        out = x @ pc
        if "vector_metadata" not in self.metadata:
            name = self.get_input_features()[0].name if self._inputs else "vec"
            cols = [OpVectorColumnMetadata((name,), (T.OPVector.type_name(),), None, None, f"pca_{i}", i)
                    for i in range(pc.shape[1])]
            self.metadata["vector_metadata"] = OpVectorMetadata(self.get_output_feature_name(), cols, {})
        return VectorColumn(out.to(v.values.dtype), self.metadata["vector_metadata"])


@register_stage
class OpPCA(UnaryEstimator):
    """Spark ``PCA(k)``: the top-k eigenvectors of the column covariance (``RowMatrix.
    computePrincipalComponentsAndExplainedVariance``); the projection does not centre the data, as Spark's. Eigen
    vectors are sign-normalised (largest-magnitude entry positive) so the fit is deterministic."""
    operation_name = "pca"
    output_type = T.OPVector
    _defaults = {"k": 2}

    def fit_columns(self, v, ds=None):
        x = _f64(v)
        n, d = x.shape
        k = int(self.params["k"])
        if not 0 < k <= d:
            raise ValueError(f"PCA k = {k} must be in [1, {d}]")
        xc = x - x.mean(0)
        cov = (xc.T @ xc) / max(n - 1, 1)
        w, vec = torch.linalg.eigh(cov)
        order = torch.argsort(w, descending=True)[:k]
        pc = vec[:, order]
        sign = torch.sign(pc.gather(0, pc.abs().argmax(0, keepdim=True)))
        pc = pc * torch.where(sign == 0, torch.ones_like(sign), sign)
        m = OpPCAModel()
        m.pc = pc
        tot = w.clamp_min(0).sum()
        m.explained_variance = (w[order].clamp_min(0) / tot) if tot > 0 else torch.zeros(k, dtype=torch.float64)
        m.params.update(self.params)
        return m
